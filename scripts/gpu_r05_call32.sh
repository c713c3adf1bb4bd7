#!/bin/bash
# round 5: state after the tail work: launch profiles, bench 512 seeds 0-2 and 4096 (driver
# protocol: 20 timed, 5 warmup), SV at 1024 / 8192 chains
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call32
mkdir -p $O
rm -f $O/summary.txt
timeout -k 10 300 python -u scripts/bench_launch_profile.py 512 20 200 5 > $O/launch_512.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/bench_launch_profile.py 4096 20 200 5 > $O/launch_4096.txt 2>&1 || exit 1
for seed in 0 1 2; do
  timeout -k 10 300 python3 bench.py --chains 512 --steps 20 --warmup 5 --seed $seed --configs none --no-cpu-baseline > $O/b512_$seed.json 2> $O/b512_$seed.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/b512_$seed.json').readline());print('512 seed $seed', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3))" >> $O/summary.txt
done
for seed in 0 1; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --seed $seed --configs none --no-cpu-baseline > $O/b4096_$seed.json 2> $O/b4096_$seed.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/b4096_$seed.json').readline());print('4096 seed $seed', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3), round(d['roofline']['frac'],4))" >> $O/summary.txt
done
timeout -k 10 300 python3 scripts/bench_configs.py sv --chains 1024 --warmup 200 --steps 10 > $O/sv1024.txt 2>&1 || exit 1
timeout -k 10 300 python3 scripts/bench_configs.py sv --chains 8192 --warmup 200 --steps 10 > $O/sv8192.txt 2>&1 || exit 1
python3 -c "
import json
for f in ('sv1024','sv8192'):
    d=[json.loads(l) for l in open('$O/'+f+'.txt') if l.startswith('{')][-1]
    print(f, d['leapfrog_per_s'], d['mean_tree'])" >> $O/summary.txt
cat $O/launch_512.txt $O/launch_4096.txt $O/summary.txt
