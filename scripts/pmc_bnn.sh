#!/bin/bash
# Kernel stats and SQ counters of the BNN potential (k_bnn, H = 69, N = 100, 2048 chains), two
# PMC passes of <= 8 SQ counters, kernel trace off (MI355X_MICROARCH.md PMC rules).
# -> gpurun_out/pmc_bnn/{stats,a,b}/ + summary.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pmc_bnn
mkdir -p "$O"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o s -- \
  python3 scripts/bench_bnn.py 69 2048 > "$O/stats.log" 2>&1 || exit $?
rm -f "$O"/stats/*kernel_trace.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/a" -o p -- \
  python3 scripts/bench_bnn.py 69 2048 > "$O/a.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU \
  SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --output-format csv -d "$O/b" -o p -- \
  python3 scripts/bench_bnn.py 69 2048 > "$O/b.log" 2>&1 || exit $?
python3 scripts/pmc_summary.py "$O" k_bnn > "$O/summary.txt"
rm -rf "$O/a" "$O/b"
