#!/bin/bash
# round 5: parity with the median-at-transition draw bound: the traced parity GPU tests and the
# c3 bench leg (BNN) that had 2 draws with a small same-chain calibration drift
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call33
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_trace.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --configs c3 > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
python3 -c "
import json
d=json.loads(open('$O/bench_c3.json').readline())
c=d['configs']['c3']; p=c.get('parity',{})
print(json.dumps({k:p.get(k) for k in ('matched','unexplained','explained','draw_drift')})[:800]); print(p.get('calibration'))"
grep -E "\[c3\]" $O/bench_c3.err | tail -8
# kernel-boundary cost micro (scripts/micro/boundary_cost.hip, built into build/abx/micro)
timeout -k 10 120 build/abx/micro/boundary_cost 2000 > $O/boundary.txt 2>&1 || exit 1
cat $O/boundary.txt
for c in 32 4096; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/bprof$c -o run -- build/abx/micro/boundary_cost 500 $c > $O/bprof$c.log 2>&1 || exit 1
  echo "== chains $c" >> $O/boundary_hist.txt
  python3 scripts/kernel_hist.py $O/bprof$c >> $O/boundary_hist.txt 2>&1 || exit 1
done
cat $O/boundary_hist.txt
