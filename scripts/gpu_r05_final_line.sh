#!/bin/bash
# round 5: the default bench line on the final HEAD (driver command)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/final_line
mkdir -p $O
timeout -k 10 1100 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 - <<PY
import json
d=json.loads(open("$O/bench.json").readline())
print("headline", round(d["value"]), round(d["roofline"]["frac"], 4), d["bench_wall_s"])
for k, c in d["configs"].items():
    p = c["parity"]
    print(k, round(c["value"]), round(c["roofline"]["frac"], 4), p["chains"], p["matched"], p.get("unexplained"), p["draw_drift"].get("geo_mean_ratio"), p["calibration"]["device_like_calibration"])
PY
