"""Average rocprofv3 counter values per dispatch of the logreg potential kernel.
usage: python scripts/pmc_summary.py <dir with a/ b/ pass outputs> [kernel name pattern]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "logreg_x3"
tot = defaultdict(float)
cnt = defaultdict(set)
for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            if pat not in row.get("Kernel_Name", ""):
                continue
            name = row["Counter_Name"]
            tot[name] += float(row["Counter_Value"])
            cnt[name].add((path, row.get("Dispatch_Id", row.get("Correlation_Id", ""))))
avg = {k: tot[k] / max(1, len(cnt[k])) for k in tot}
for k in sorted(avg):
    print(f"{k:32s} {avg[k]:.6g}  (dispatches {len(cnt[k])})")
w = avg.get("SQ_WAVE_CYCLES")
if w:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
              "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_MISC"):
        if k in avg:
            print(f"{k} / WAVE_CYCLES = {avg[k] / w:.3f}")
if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
    # SQ_VALU_MFMA_BUSY_CYCLES counts cycles (32 per 32x32x16 bf16 MFMA, MI355X_MICROARCH.md)
    # summed over SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs: kernel cycles = GRBM / 8
    busy = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
    print(f"MFMA pipe busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCD x 1024 SIMD) = {busy:.3f}")
