# A/B of library builds on the SV config (fused wide step): per-rank share at N=8 and one GPU.
# usage: bash scripts/ab_sv.sh "VARIANTS" "CHAINS"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for ch in $2; do for v in $1; do
  timeout -k 10 200 python3 scripts/bench_configs.py sv --chains $ch --warmup 50 --steps 20 --lib build/ab/$v/libnumpyro_amd.so > gpurun_out/sv_${v}_${ch}.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/sv_${v}_${ch}.json').read().strip().splitlines()[-1]); print('$ch $v', round(d['leapfrog_per_s']), d.get('mean_tree_size'))" >> gpurun_out/ab_sv.txt
done; done
