"""Per-launch HBM bytes of the covtype potential inside the bench's timed region, from the
FETCH_SIZE / WRITE_SIZE passes of scripts/pmc_bench_traffic.sh (MI355X_MICROARCH.md HBM section:
FETCH_SIZE in KB doubled on gfx950, WRITE_SIZE in KB as is).  The timed launches are the last
`leapfrog_launches` dispatches of each potential kernel (x3 main or tail form, finalize).
usage: python scripts/bench_traffic_summary.py gpurun_out/traffic_bench > summary.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]


def line(log):
    for ln in open(log):
        if ln.startswith("{"):
            d = json.loads(ln)
    return d


def per_dispatch(d, counter):
    """{dispatch id: (kernel kind, bytes)} for the potential kernels"""
    vals = defaultdict(float)
    kind = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] != counter:
                    continue
                k = row["Kernel_Name"]
                if "k_logreg_x3" in k:
                    kk = "x3"
                elif "k_logreg_finalize" in k:
                    kk = "finalize"
                else:
                    continue
                did = int(row.get("Dispatch_Id") or row.get("Correlation_Id"))
                vals[did] += float(row["Counter_Value"])
                kind[did] = kk
    return vals, kind


out = {}
for counter, sub, scale in (("FETCH_SIZE", "f", 2.0 * 1024), ("WRITE_SIZE", "w", 1024.0)):
    ln = line(os.path.join(root, sub + ".log"))
    n = int(ln["leapfrog_launches"])
    vals, kind = per_dispatch(os.path.join(root, sub), counter)
    for kk in ("x3", "finalize"):
        ids = sorted(i for i in vals if kind[i] == kk)[-n:]
        out[f"{kk}_{counter}_bytes_per_launch"] = sum(vals[i] for i in ids) * scale / len(ids)
    out[f"{sub}_run_leapfrog_launches"] = n
    out[f"{sub}_run_value"] = ln["value"]
rd = out["x3_FETCH_SIZE_bytes_per_launch"] + out["finalize_FETCH_SIZE_bytes_per_launch"]
wr = out["x3_WRITE_SIZE_bytes_per_launch"] + out["finalize_WRITE_SIZE_bytes_per_launch"]
out["hbm_bytes_per_launch"] = rd + wr
print(json.dumps(out, indent=1))
