# A/B of library builds on the covtype bench over several seeds (the timed region's straggler
# chains differ with the trajectories).  usage: bash scripts/ab_seeds.sh CHAINS "SEEDS" "VARIANTS"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for sd in $2; do for v in $3; do
  o=gpurun_out/abs_${v}_$1_$sd.json
  timeout -k 10 150 python3 bench.py --chains $1 --seed $sd --steps 20 --warmup 5 --no-cpu-baseline --configs none --lib build/ab/$v/libnumpyro_amd.so > $o 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('$o').read().strip().splitlines()[-1]); print('$1 seed $sd $v', round(d['value']), round(d['mean_tree_size'],3), round(d['ms_per_step'],2))" >> gpurun_out/ab_seeds.txt
done; done
