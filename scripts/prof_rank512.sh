#!/bin/bash
# Kernel trace of one rank's share at 8 GPUs (bench.py --chains 512 on one GPU), summarised
# on the box (per-kernel stats + the potential launches by duration); the trace itself is
# dropped (too large to copy back).  usage: bash scripts/prof_rank512.sh [chains]
set -o pipefail
n=${1:-512}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/k$n
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O" -o k -- \
  python3 bench.py --no-cpu-baseline --chains "$n" > "$O/bench.log" 2>&1 || exit $?
python3 - "$O" > "$O/summary.txt" <<'EOF'
import csv, sys
import numpy as np
o = sys.argv[1]
for x in list(csv.DictReader(open(f"{o}/k_kernel_stats.csv")))[:6]:
    print(x["Name"][:70], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1), x["Percentage"])
t = [x for x in csv.DictReader(open(f"{o}/k_kernel_trace.csv")) if "logreg_x3" in x["Kernel_Name"]]
d = np.array([(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3 for x in t])
print("x3 launches", len(d), "total ms", round(d.sum() / 1e3, 1))
for lo, hi in [(0, 140), (140, 200), (200, 300), (300, 450), (450, 1e9)]:
    m = (d >= lo) & (d < hi)
    print(f"  {lo}-{hi} us: {m.sum()} launches, {d[m].sum() / 1e3:.1f} ms")
EOF
rm -f "$O/k_kernel_trace.csv"
