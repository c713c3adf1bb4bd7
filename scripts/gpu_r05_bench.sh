#!/bin/bash
# round 5: the default bench line (headline + configs 2-4 with CPU baselines and parity legs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${BENCH_TAG:-bench}
mkdir -p $O
timeout -k 10 1100 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 - <<PY
import json
d = json.loads(open("$O/bench.json").readline())
print("headline", round(d["value"]), d["roofline"]["frac"], d["ms_per_step"])
for k, c in d.get("configs", {}).items():
    r = c.get("roofline", {})
    print(k, round(c["value"]), round(r.get("frac", 0), 4), (r.get("valu") or {}).get("frac"), c.get("max_split_rhat"))
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"].get("kind"))
print("parity", json.dumps(d.get("parity", {}))[:400])
PY
