#!/bin/bash
# Chain groups on their own streams (Engine.chain_groups) on the headline at one rank's share of
# 8 GPUs (512 chains) and at 4096 chains.
run() { echo "== $*"; python -u bench.py --configs none --no-cpu-baseline "$@" 2>&1 | grep '^{' || exit 1; }
for g in "$@"; do
  run --chains 512 --chain-groups $g
done
for g in "$@"; do
  run --chains 4096 --chain-groups $g
done
