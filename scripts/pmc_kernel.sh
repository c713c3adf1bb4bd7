#!/bin/bash
# SQ counters of one covtype potential variant (scripts/bench_potential.py, C=4096), two
# passes of <= 8 SQ counters each, kernel trace off (MI355X_MICROARCH.md PMC rules).
# usage: bash scripts/pmc_kernel.sh <variant> <tag>  -> gpurun_out/pmc_<tag>/{a,b}/
set -o pipefail
v=${1:-19}; tag=${2:-v$v}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pmc_$tag
mkdir -p "$O"
[ "$v" = d ] && unset NMX_LOGREG_VARIANT || export NMX_LOGREG_VARIANT=$v
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/a" -o p -- \
  python3 scripts/bench_potential.py "$v" 4096 > "$O/a.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_COEXEC_CYCLES \
  SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES --output-format csv -d "$O/b" -o p -- \
  python3 scripts/bench_potential.py "$v" 4096 > "$O/b.log" 2>&1 || exit $?
pat=logreg_x3; case $v in 30|31|32|d) ;; *) pat=logreg_rowlanes;; esac
python3 scripts/pmc_summary.py "$O" $pat > "$O/summary.txt"
