#!/bin/bash
# k_gemm_x3 chain tile: 64 chains per workgroup (build/ab/ct2) vs 128 (build/ab/ct4, one
# workgroup per CU, 1.5x MFMA work per staged byte): dense tests on ct4, the product alone, and
# the dense-mass wide configs (c2 funnel-10k, c3 BNN) pooled.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in ct4 ct4b3; do NUMPYRO_AMD_LIB=build/ab/$v/libnumpyro_amd.so timeout -k 10 300 python -u -m pytest -q --timeout 200 \
  --timeout-method thread -m gpu tests/test_gpu_dense.py > gpurun_out/${v}_tests.txt 2>&1 || exit 1; done
bash scripts/ab_gemm.sh "ct2 ct4 ct4b3" "10000:4096 10000:2048 5038:2048" || exit 1
run() { echo "== $*"; timeout -k 10 200 python -u scripts/bench_configs.py "$@" 2>&1 | grep '^{' || exit 1; }
for v in ct2 ct4 ct4b3; do
  run funnel --chains 4096 --warmup 30 --steps 5 --lib build/ab/$v/libnumpyro_amd.so
  run bnn --chains 2048 --warmup 30 --steps 5 --lib build/ab/$v/libnumpyro_amd.so
done
