"""Per-kernel duration histogram from a rocprofv3 --kernel-trace run (csv).

    python scripts/kernel_hist.py <rocprof dir> [name substring ...]

For each kernel (matching the substrings, all if none): dispatches, total ms, and the
duration quantiles (us), plus the mean gap between consecutive dispatches on the queue."""
import collections
import csv
import glob
import sys

import numpy as np

root, pats = sys.argv[1], sys.argv[2:]
rows = []
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if pats and not any(p in n for p in pats):
        continue
    by[n[:90]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    d = np.array(d)
    q = np.percentile(d, [10, 50, 90, 99])
    print(f"{n:90s} n={len(d):6d} total={d.sum() / 1e3:9.2f} ms  p10/50/90/99 = "
          f"{q[0]:8.1f} {q[1]:8.1f} {q[2]:8.1f} {q[3]:8.1f} us")
# busy vs span over the last timed region: gaps between consecutive dispatches
st = np.array([int(r["Start_Timestamp"]) for r in rows])
en = np.array([int(r["End_Timestamp"]) for r in rows])
if len(st) > 1:
    gap = (st[1:] - en[:-1]) / 1e3
    print(f"dispatches {len(st)}, gap p50 {np.median(gap):.1f} us, p90 {np.percentile(gap, 90):.1f} us")
