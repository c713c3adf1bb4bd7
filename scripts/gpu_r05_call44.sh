#!/bin/bash
# round 5: fused covtype step as 4-wave blocks of 8 chains (NV = 32 lanes per chain as before,
# so bitwise the same draws) vs 8-wave blocks of 16: bitwise check, 512 / 4096-chain bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call44
mkdir -p $O
rm -f $O/summary.txt
timeout -k 10 600 python3 -u scripts/step_ab.py numpyro_amd/_lib/libnumpyro_amd.so build/abx/step48/libnumpyro_amd.so > $O/step_ab.txt 2>&1 || { cat $O/step_ab.txt; exit 1; }
cat $O/step_ab.txt
for v in head step48; do
  L=numpyro_amd/_lib/libnumpyro_amd.so; [ $v = step48 ] && L=build/abx/step48/libnumpyro_amd.so
  for seed in 0 2; do
    timeout -k 10 300 python3 bench.py --chains 512 --steps 20 --warmup 5 --seed $seed --configs none --no-cpu-baseline --lib $L > $O/b512_${v}_$seed.json 2> $O/b512_${v}_$seed.err || exit 1
    python3 -c "import json;d=json.loads(open('$O/b512_${v}_$seed.json').readline());print('$v 512 seed $seed', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3))" >> $O/summary.txt
  done
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --configs none --no-cpu-baseline --lib $L > $O/b4096_$v.json 2> $O/b4096_$v.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/b4096_$v.json').readline());print('$v 4096', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3), round(d['roofline']['frac'],4))" >> $O/summary.txt
done
cat $O/summary.txt
