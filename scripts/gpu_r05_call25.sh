#!/bin/bash
# round 5: fused-step variants (CPW 8, batched rows) vs base: per-kernel durations in the
# covtype 512-chain protocol, plus bench --chains 512 seeds 0/1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call25
mkdir -p $O
rm -f $O/summary.txt
for v in base cpw8 lr2; do
  L=$PWD/build/abx/$v/libnumpyro_amd.so; [ $v = base ] && L=$PWD/numpyro_amd/_lib/libnumpyro_amd.so
  export NUMPYRO_AMD_LIB=$L
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/bench_launch_profile.py 512 20 200 5 > $O/launch_$v.txt 2>&1 || exit 1
  echo "== $v" >> $O/summary.txt
  head -2 $O/launch_$v.txt | tail -1 >> $O/summary.txt
  python3 scripts/kernel_hist.py $O/kt_$v nuts_step finalize >> $O/summary.txt || exit 1
  rm -rf $O/kt_$v
  for seed in 0 1; do
    timeout -k 10 300 python3 bench.py --chains 512 --steps 20 --warmup 5 --seed $seed --configs none --no-cpu-baseline > $O/b_${v}_$seed.json 2> $O/b_${v}_$seed.err || exit 1
    python3 -c "import json;d=json.loads(open('$O/b_${v}_$seed.json').readline());print('$v seed $seed', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3))" >> $O/summary.txt
  done
done
unset NUMPYRO_AMD_LIB
cat $O/summary.txt
