#!/bin/bash
# Persistent wide kernel after the single-level checkpoint preload: rows in flight (NMX_PX_B) x
# waves per SIMD the kernel is compiled for (NMX_PX_OCC), library variants of scripts/ab_build.py.
run() { echo "== $*"; python -u scripts/bench_configs.py "$@" 2>&1 | grep '^{' || exit 1; }
for v in "$@"; do
  L=build/ab/$v/libnumpyro_amd.so
  [ "$v" = cur ] && L=numpyro_amd/_lib/libnumpyro_amd.so
  run sv --chains 8192 --warmup 50 --steps 10 --lib $L
  run sv --chains 1024 --warmup 50 --steps 10 --lib $L
  NMX_PERSIST_NT=256 run funnel --dense 0 --chains 4096 --warmup 30 --steps 10 --lib $L
  NMX_PERSIST_NT=512 run funnel --dense 0 --chains 4096 --warmup 30 --steps 10 --lib $L
done
