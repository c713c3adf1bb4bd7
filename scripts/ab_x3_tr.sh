#!/bin/bash
# covtype main kernel with GEMM2 from transposed reads (build/ab/x3tr, -DNMX_X3_TR=1) vs current.
run() { echo "== $*"; python -u bench.py --configs none --no-cpu-baseline "$@" 2>&1 | grep '^{' || exit 1; }
run --chains 512
run --chains 512 --lib build/ab/x3tr/libnumpyro_amd.so
run --chains 4096
run --chains 4096 --lib build/ab/x3tr/libnumpyro_amd.so
