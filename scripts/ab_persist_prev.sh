#!/bin/bash
# Persistent wide kernel: current vs a previous build (build/ab/prevsc).
run() { echo "== $*"; python -u scripts/bench_configs.py "$@" 2>&1 | grep '^{' || exit 1; }
for L in numpyro_amd/_lib/libnumpyro_amd.so build/ab/prevsc/libnumpyro_amd.so; do
  run sv --chains 8192 --warmup 50 --steps 10 --lib $L
  run sv --chains 1024 --warmup 50 --steps 10 --lib $L
  run funnel --dense 0 --chains 4096 --warmup 30 --steps 10 --lib $L
done
