#!/bin/bash
# Persistent wide kernel A/B: threads per chain (NMX_PERSIST_NT) and rows in flight per thread
# (library variants built by scripts/ab_build.py with -DNMX_PX_B=..).
run() { echo "== $*"; python -u scripts/bench_configs.py "$@" 2>&1 | grep '^{' || exit 1; }
for nt in 128 256 512; do
  NMX_PERSIST_NT=$nt run sv --chains 8192 --warmup 50 --steps 10
  NMX_PERSIST_NT=$nt run sv --chains 1024 --warmup 50 --steps 10
  NMX_PERSIST_NT=$nt run funnel --dense 0 --chains 4096 --warmup 30 --steps 5
done
for v in pb1 pb3; do
  NMX_PERSIST_NT=256 run sv --chains 8192 --warmup 50 --steps 10 --lib build/ab/$v/libnumpyro_amd.so
  NMX_PERSIST_NT=512 run funnel --dense 0 --chains 4096 --warmup 30 --steps 5 --lib build/ab/$v/libnumpyro_amd.so
done
