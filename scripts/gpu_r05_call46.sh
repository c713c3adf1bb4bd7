#!/bin/bash
# round 5: C NUTS restatement with per-thread chain loops for per-chain potentials (SV probe)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call46
mkdir -p $O
for i in 1 2; do timeout -k 10 120 python3 scripts/sv_cpu_share.py >> $O/perthread.txt 2>&1 || exit 1; done
cat $O/perthread.txt
timeout -k 10 1100 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 - <<PY
import json
d=json.loads(open("$O/bench.json").readline())
print("headline", round(d["value"]), round(d["roofline"]["frac"], 4), d["bench_wall_s"], "cpu", round(d["cpu_baseline"]["value"]), round(d["cpu_baseline"]["potential_share"], 3))
for k, c in d["configs"].items():
    p = c["parity"]; cb = c["cpu_baseline"]
    print(k, round(c["value"]), round(c["roofline"]["frac"], 4), "cpu", round(cb["value"], 1), round(cb["potential_share"], 3), "par", p["chains"], p["matched"], p.get("unexplained"), p["draw_drift"].get("geo_mean_ratio"), p["calibration"]["device_like_calibration"])
PY
