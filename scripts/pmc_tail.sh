#!/bin/bash
# SQ counters of the covtype potential in tail launches (16 active chains of 4096), two passes
# of <= 8 SQ counters, kernel trace off.  usage: bash scripts/pmc_tail.sh [count]
set -o pipefail
n=${1:-16}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pmc_tail
mkdir -p "$O"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS --output-format csv -d "$O/a" -o p -- \
  python3 scripts/logreg_list_bench.py 36 $n > "$O/a.log" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU \
  SQ_WAVES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC --output-format csv -d "$O/b" -o p -- \
  python3 scripts/logreg_list_bench.py 36 $n > "$O/b.log" 2>&1 || exit $?
python3 scripts/pmc_summary.py "$O" logreg_x3 > "$O/summary.txt"
rm -rf "$O/a" "$O/b"
