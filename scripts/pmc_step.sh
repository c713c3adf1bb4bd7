#!/bin/bash
# SQ counters of the fused NUTS step kernel inside a short covtype bench run (two passes of
# <= 8 SQ counters, kernel trace off).  usage: bash scripts/pmc_step.sh <tag>
set -o pipefail
tag=${1:-step}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pmc_$tag
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS --output-format csv -d "$O/a" -o p -- \
  python3 bench.py --no-cpu-baseline --steps 5 --warmup 5 > "$O/a.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS \
  SQ_INSTS_SMEM SQ_WAVES SQ_INST_CYCLES_VMEM --output-format csv -d "$O/b" -o p -- \
  python3 bench.py --no-cpu-baseline --steps 5 --warmup 5 > "$O/b.log" 2>&1 || exit $?
python3 scripts/pmc_summary.py "$O" k_nuts_step > "$O/summary.txt"
