"""Average duration of the covtype potential kernels over the bench's TIMED launches, from a
rocprofv3 --kernel-trace CSV of `bench.py` (the trace also holds warmup launches, which the
stats summary averages in): the last `leapfrog_launches` dispatches of each kernel.
usage: python scripts/trace_timed_avg.py <kernel_trace.csv> <bench_line.json>"""
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
line = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
n = int(line["leapfrog_launches"])
out = {"timed_launches": n, "bench_potential_ms_per_launch": line["potential_ms_per_launch"]}
total = 0.0
for key in ("logreg_x3", "logreg_finalize"):
    k = sorted((r for r in rows if key in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))[-n:]
    ms = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in k) / len(k) / 1e6
    out[f"{key}_ms_avg"] = ms
    total += ms
out["trace_potential_ms_per_launch"] = total
out["relative_difference"] = total / line["potential_ms_per_launch"] - 1.0
print(json.dumps(out, indent=1))
