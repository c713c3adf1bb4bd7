#!/bin/bash
# The persistent wide schedule (nmx_nuts_run_wide) against the launched fused step on SV and the
# funnel with diagonal mass, and the persistent kernel's threads per chain (NMX_PERSIST_NT).
# usage: scripts/ab_persist.sh [nt ...]
run() { echo "== $*"; python -u scripts/bench_configs.py "$@" 2>&1 | grep '^{' || exit 1; }
for ch in 1024 8192; do
  run sv --chains $ch --warmup 50 --steps 10 --fused
  run sv --chains $ch --warmup 50 --steps 10
  for nt in "$@"; do NMX_PERSIST_NT=$nt run sv --chains $ch --warmup 50 --steps 10; done
done
run funnel --dense 0 --chains 4096 --warmup 30 --steps 5 --fused
run funnel --dense 0 --chains 4096 --warmup 30 --steps 5
for nt in "$@"; do NMX_PERSIST_NT=$nt run funnel --dense 0 --chains 4096 --warmup 30 --steps 5; done
