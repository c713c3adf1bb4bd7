#!/bin/bash
# Dense-mass wide configs: the per-chain step on a chain-row arena (k_chain_step) vs the D-slice
# kernels (--slices), funnel-10k pooled (c2 shape) and BNN H=69 pooled (c3 shape).
run() { echo "== $*"; python -u scripts/bench_configs.py "$@" 2>&1 | grep '^{' || exit 1; }
run funnel --chains 4096 --warmup 30 --steps 5
run funnel --chains 4096 --warmup 30 --steps 5 --slices
run bnn --chains 2048 --warmup 30 --steps 5
run bnn --chains 2048 --warmup 30 --steps 5 --slices
