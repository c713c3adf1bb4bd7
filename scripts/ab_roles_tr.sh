#!/bin/bash
# covtype tail form with GEMM2 operands from transposed reads of the GEMM1 image (current) vs the
# previous tail form that streams the B pieces (build/ab/oldroles), at 512 and 4096 chains.
run() { echo "== $*"; python -u bench.py --configs none --no-cpu-baseline "$@" 2>&1 | grep '^{' || exit 1; }
run --chains 512
run --chains 512 --lib build/ab/oldroles/libnumpyro_amd.so
run --chains 4096
run --chains 4096 --lib build/ab/oldroles/libnumpyro_amd.so
