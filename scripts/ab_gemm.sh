# A/B of library builds on the split-bf16 chain products (k_gemm_x3, all three triangles).
# usage: bash scripts/ab_gemm.sh "G0 G4" "10000:4096 5038:2048"   -> gpurun_out/ab_gemm.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for dc in $2; do for v in $1; do
  echo "== $v D:C=$dc" >> gpurun_out/ab_gemm.txt
  timeout -k 10 120 python3 scripts/bench_configs.py gemm ${dc%%:*} ${dc##*:} --lib build/ab/$v/libnumpyro_amd.so 2>/dev/null | grep k_gemm_x3 >> gpurun_out/ab_gemm.txt || exit 1
done; done
