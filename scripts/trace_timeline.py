"""GPU timeline of the bench's timed region from a rocprofv3 --kernel-trace CSV: the window from
the first to the last of the final `leapfrog_launches` potential dispatches; per-kernel time,
GPU busy time (union of kernel intervals) and idle gaps.
usage: python scripts/trace_timeline.py <kernel_trace.csv> <bench_line.json> [potential kernel key]"""
import csv
import json
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
line = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
key = sys.argv[3] if len(sys.argv) > 3 else "logreg_x3"
n = int(line["leapfrog_launches"])
pot = sorted((r for r in rows if key in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))[-n:]
t0, t1 = int(pot[0]["Start_Timestamp"]), int(pot[-1]["End_Timestamp"])
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows
            if int(r["Start_Timestamp"]) >= t0 and int(r["End_Timestamp"]) <= t1)
per = defaultdict(lambda: [0, 0.0])
busy, cur_s, cur_e = 0, None, None
for s, e, name in iv:
    m = re.search(r"(k_\w+|__amd\w+|at::native::\w+)", name)
    short = m.group(1) if m else name[:48]
    per[short][0] += 1
    per[short][1] += (e - s) / 1e6
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None:
    busy += cur_e - cur_s
span = (t1 - t0) / 1e6
durs = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in pot)
hist = {}
for lo, hi in ((0, 50), (50, 100), (100, 150), (150, 200), (200, 300), (300, 500), (500, 1000), (1000, 1e9)):
    sel = [d for d in durs if lo <= d < hi]
    hist[f"{lo}-{hi if hi < 1e9 else 'inf'}us"] = {"launches": len(sel), "ms": round(sum(sel) / 1e3, 2)}
out = {"potential_duration_histogram": hist, "window_ms": span, "gpu_busy_ms": busy / 1e6, "idle_frac": 1 - busy / 1e6 / span, "timed_launches": n,
       "kernels": {k: {"calls": c, "ms": round(ms, 3), "avg_us": round(1e3 * ms / c, 2)} for k, (c, ms) in
                   sorted(per.items(), key=lambda kv: -kv[1][1])}}
print(json.dumps(out, indent=1))
