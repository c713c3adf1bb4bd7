#!/bin/bash
# round 5: LDS-only step barriers + batched rows + branch-free finalize z loads: GPU suite,
# stamps, kernel durations, bench --chains 512 seeds 0-2 and the 4096 headline protocol
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call27
mkdir -p $O
export PYTHONUNBUFFERED=1
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.txt 2>&1
rc=$?
tail -2 $O/tests.txt
grep -E "FAILED|ERROR" $O/tests.txt | head
[ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u scripts/step_stamps.py build/abx/stepst/libnumpyro_amd.so 512 20 > $O/step.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/fin_stamps.py build/abx/finst/libnumpyro_amd.so 1 > $O/fin.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 scripts/bench_launch_profile.py 512 20 200 5 > $O/launch_512.txt 2>&1 || exit 1
python3 scripts/kernel_hist.py $O/kt logreg nuts_step > $O/hist_512.txt || exit 1
rm -rf $O/kt
for seed in 0 1 2; do
  timeout -k 10 300 python3 bench.py --chains 512 --steps 20 --warmup 5 --seed $seed --configs none --no-cpu-baseline > $O/b512_$seed.json 2> $O/b512_$seed.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/b512_$seed.json').readline());print('512 seed $seed', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3))" >> $O/summary.txt
done
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --configs none --no-cpu-baseline > $O/b4096.json 2> $O/b4096.err || exit 1
python3 -c "import json;d=json.loads(open('$O/b4096.json').readline());print('4096', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3), round(d['roofline']['frac'],4))" >> $O/summary.txt
cat $O/step.txt $O/fin.txt $O/hist_512.txt $O/summary.txt
