#!/bin/bash
# covtype potential: the role-split kernel (k_logreg_x3_roles) for launches of up to
# NMX_X3_TAIL_TILES 128-chain tiles, at one rank's share of 8 GPUs (512 chains).
run() { echo "== $*"; python -u bench.py --configs none --no-cpu-baseline "$@" 2>&1 | grep '^{' || exit 1; }
run --chains 512
for v in "$@"; do run --chains 512 --lib build/ab/$v/libnumpyro_amd.so; done
