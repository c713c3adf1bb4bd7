#!/bin/bash
# k_gemm_x3 workgroup tile A/B: build/ab/<variant> libraries (ct2 = 128 rows x 64 chains, 4 waves,
# two workgroups per CU -- the default; ct4 = 128 x 128, one workgroup per CU; r8c4 = 256 x 128,
# 8 waves).  Dense tests on every non-default variant, the product alone, then the dense-mass
# wide configs (c2 funnel-10k, c3 BNN) pooled.   usage: scripts/ab_gemm_ct.sh "ct2 r8c4"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=${1:-"ct2 ct4"}
for v in $V; do [ "$v" = ct2 ] && continue
  NUMPYRO_AMD_LIB=build/ab/$v/libnumpyro_amd.so timeout -k 10 300 python -u -m pytest -q --timeout 200 \
    --timeout-method thread -m gpu tests/test_gpu_dense.py > gpurun_out/${v}_tests.txt 2>&1 || exit 1
done
bash scripts/ab_gemm.sh "$V" "10000:4096 10000:2048 5038:2048" || exit 1
run() { echo "== $*"; timeout -k 10 200 python -u scripts/bench_configs.py "$@" 2>&1 | grep '^{' || exit 1; }
for v in $V; do
  run funnel --chains 4096 --warmup 30 --steps 5 --lib build/ab/$v/libnumpyro_amd.so
  run bnn --chains 2048 --warmup 30 --steps 5 --lib build/ab/$v/libnumpyro_amd.so
done
