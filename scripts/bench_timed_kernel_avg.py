"""Average duration of the covtype potential kernels over the bench's timed launches, from a
rocprofv3 --kernel-trace run of `bench.py --configs none --no-cpu-baseline`: the last
`leapfrog_launches` dispatches of k_logreg_x3 (main or tail form) and of k_logreg_finalize, to
check against the bench line's in-run HIP-event figure (`potential_ms_per_launch`).
usage: python scripts/bench_timed_kernel_avg.py <rocprof dir> <bench stdout log>"""
import csv
import glob
import json
import os
import sys

root, log = sys.argv[1], sys.argv[2]
line = [json.loads(ln) for ln in open(log) if ln.startswith("{")][-1]
n = int(line["leapfrog_launches"])
rows = []
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
out = {"leapfrog_launches": n, "bench_potential_ms_per_launch": line.get("potential_ms_per_launch")}
tot = 0.0
for kk, pat in (("x3", "k_logreg_x3"), ("finalize", "k_logreg_finalize")):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if pat in r["Kernel_Name"]][-n:]
    out[f"{kk}_ms_avg"] = sum(d) / len(d)
    tot += out[f"{kk}_ms_avg"]
out["trace_potential_ms_per_launch"] = tot
b = out["bench_potential_ms_per_launch"]
if b:
    out["trace_vs_bench"] = tot / b - 1.0
print(json.dumps(out, indent=1))
