#!/bin/bash
# round 5, final HEAD: one rank's share at 8 GPUs (512 covtype chains, seeds 0-2, driver protocol
# 20 timed / 5 warmup) and SV at 1024 chains
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/perrank
mkdir -p $O
rm -f $O/summary.txt
for seed in 0 1 2; do
  timeout -k 10 300 python3 bench.py --chains 512 --steps 20 --warmup 5 --seed $seed --configs none --no-cpu-baseline > $O/b512_$seed.json 2> $O/b512_$seed.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/b512_$seed.json').readline());print('covtype 512 seed $seed', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3), round(d['roofline']['frac'],4))" >> $O/summary.txt
done
timeout -k 10 300 python3 scripts/bench_configs.py sv --chains 1024 --warmup 200 --steps 10 > $O/sv1024.txt 2>&1 || exit 1
python3 -c "
import json
d=[json.loads(l) for l in open('$O/sv1024.txt') if l.startswith('{')][-1]
print('SV 1024', d['leapfrog_per_s'], d['wall_s'], d['mean_tree'])" >> $O/summary.txt
cat $O/summary.txt
