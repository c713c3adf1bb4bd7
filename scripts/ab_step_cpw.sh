#!/bin/bash
# covtype fused step: 16 chains per wave (32 lanes per chain, build/ab/cpw16) vs 8 (64 lanes per
# chain, twice the blocks: build/ab/cpw8), at the 8-GPU share (512 chains) and at 4096.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
run() { echo "== $*"; timeout -k 10 200 python -u bench.py --configs none --no-cpu-baseline "$@" 2>&1 | grep '^{' || exit 1; }
for v in cpw16 cpw8 cpw16 cpw8; do run --chains 512 --lib build/ab/$v/libnumpyro_amd.so; done
for v in cpw16 cpw8; do run --chains 4096 --lib build/ab/$v/libnumpyro_amd.so; done
