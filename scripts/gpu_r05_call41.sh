#!/bin/bash
# round 5: the c3 parity leg over 16 chains x 2 transitions (20 -> ~40 paired drifts)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call41
mkdir -p $O
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --configs c3 > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
python3 -c "
import json
d=json.loads(open('$O/bench_c3.json').readline())
c=d['configs']['c3']; p=c['parity']
print(round(c['value']), d['bench_wall_s'], p.get('reference_seconds'), {k:p.get(k) for k in ('chains','matched','unexplained','kinds')}, p['draw_drift'], p['calibration'])"
