#!/bin/bash
# Kernel stats and PMC counters of the dense whitening product k_gemm_x3 (D = 10000 upper
# triangle, 4096 chains (config 2)): separate passes of <= 8 SQ / <= 4 TCC counters, no trace domains.
# -> gpurun_out/pmc_gemm/{stats,...} + summary.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/pmc_gemm
mkdir -p "$O"
B="python3 scripts/bench_gemm_x3.py 10000 4096 5"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o s -- $B > "$O/stats.log" 2>&1 || exit $?
rm -f "$O"/stats/*kernel_trace.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/a" -o p -- $B > "$O/a.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU \
  SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --output-format csv -d "$O/b" -o p -- $B > "$O/b.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/c" -o p -- $B > "$O/c.log" 2>&1 || exit $?
python3 scripts/pmc_summary.py "$O" k_gemm_x3 > "$O/summary.txt"
cat "$O/summary.txt"
