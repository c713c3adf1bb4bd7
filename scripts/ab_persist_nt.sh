#!/bin/bash
# Threads per chain of the persistent wide kernel (NMX_PERSIST_NT) at the current defaults.
run() { echo "== $*"; python -u scripts/bench_configs.py "$@" 2>&1 | grep '^{' || exit 1; }
for nt in "$@"; do
  NMX_PERSIST_NT=$nt run sv --chains 8192 --warmup 50 --steps 10
  NMX_PERSIST_NT=$nt run sv --chains 1024 --warmup 50 --steps 10
  NMX_PERSIST_NT=$nt run funnel --dense 0 --chains 4096 --warmup 30 --steps 10
done
