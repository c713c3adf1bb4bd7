#!/bin/bash
# round 5 A/B: k_bnn LDS swizzle (r04 source vs now, bitwise + timing), covtype split count S
# (256 / 192 / 128) on the launch-vs-active curve and bench --chains 512 / 4096
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/ab3
mkdir -p $O
export PYTHONUNBUFFERED=1
A=build/abx
timeout -k 10 300 python -u scripts/ab_bnn.py $A/bnn_r04/libnumpyro_amd.so $A/bnn_new/libnumpyro_amd.so > $O/bnn.txt 2>&1 || exit 1
cat $O/bnn.txt
for v in bnn_new s192 s128; do
  timeout -k 10 200 python -u scripts/logreg_list_bench.py 1,32,128,256,257,512,1024,2048,4096 $A/$v/libnumpyro_amd.so > $O/list_$v.txt 2>&1 || exit 1
  echo "== $v"; cat $O/list_$v.txt
done
for v in bnn_new s192 s128; do
  for seed in 0 1; do
    timeout -k 10 240 python -u bench.py --lib $A/$v/libnumpyro_amd.so --chains 512 --configs none --no-cpu-baseline --steps 20 --warmup 5 --seed $seed > $O/b512_${v}_s$seed.json 2> $O/b512_${v}_s$seed.err || exit 1
    python3 -c "import json;d=json.load(open('$O/b512_${v}_s$seed.json'));print('$v 512 seed $seed', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3), round(d['roofline']['frac'],4))"
  done
  timeout -k 10 240 python -u bench.py --lib $A/$v/libnumpyro_amd.so --configs none --no-cpu-baseline --steps 20 --warmup 5 > $O/b4096_$v.json 2> $O/b4096_$v.err || exit 1
  python3 -c "import json;d=json.load(open('$O/b4096_$v.json'));print('$v 4096', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3), round(d['roofline']['frac'],4))"
done
