"""VALU issue summary of one kernel from a rocprofv3 --pmc --kernel-trace run.

    python scripts/valu_summary.py <rocprof dir> <bench_configs log> <kernel name substring>

Sums the kernel's counters over its dispatches, takes its durations from the kernel trace and
the chain-leapfrogs from the bench_configs JSON line (warmup + timed), and prints the VALU
wave-instructions per chain-leapfrog, the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / busy
time, MI355X_MICROARCH.md 'DVFS give-back') and the issue fraction against the SIMDs' peak of
one wave64 VALU instruction per 2 cycles (256 CUs x 4 SIMDs), as JSON.
"""
import collections
import csv
import glob
import json
import sys

root, log, name = sys.argv[1:4]
tot = collections.defaultdict(float)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if name in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
ns = 0.0
n = 0
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if name in r["Kernel_Name"]:
            ns += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            n += 1
rec = [json.loads(x) for x in open(log) if x.startswith("{")][-1]
leap = rec["leapfrogs"] + rec["warmup_leapfrogs"]
sec = ns * 1e-9
clock = tot["GRBM_GUI_ACTIVE"] / 8 / sec if sec > 0 else float("nan")
per = tot["SQ_INSTS_VALU"] / leap
rate = tot["SQ_INSTS_VALU"] / sec
peak = 256 * 4 * 0.5 * clock
out = {"kernel": name, "dispatches": n, "kernel_s": sec, "chain_leapfrogs": leap,
       "valu_wave_insts_per_leapfrog": per, "salu_per_leapfrog": tot["SQ_INSTS_SALU"] / leap,
       "effective_clock_ghz": clock / 1e9, "valu_issue_rate": rate, "valu_issue_peak": peak,
       "valu_issue_frac": rate / peak, "counters": dict(tot), "bench": rec}
print(json.dumps(out, indent=1))
