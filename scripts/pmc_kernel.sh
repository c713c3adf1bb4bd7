#!/bin/bash
# SQ counters of the covtype potential (scripts/bench_potential.py, C=4096), two passes of
# <= 8 SQ counters each, kernel trace off (MI355X_MICROARCH.md PMC rules).
# usage: bash scripts/pmc_kernel.sh <ignored> <tag>  -> gpurun_out/pmc_<tag>/{a,b}/
set -o pipefail
v=${1:-d}; tag=${2:-x3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pmc_$tag
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/a" -o p -- \
  python3 scripts/bench_potential.py "$v" 4096 > "$O/a.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_COEXEC_CYCLES \
  SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES --output-format csv -d "$O/b" -o p -- \
  python3 scripts/bench_potential.py "$v" 4096 > "$O/b.log" 2>&1 || exit $?
python3 scripts/pmc_summary.py "$O" logreg_x3 > "$O/summary.txt"
