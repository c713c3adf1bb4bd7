#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE: separate passes) and SQ counters of the wide NUTS step
# kernels in the funnel-10k diag config.  usage: bash scripts/pmc_wide.sh <tag> [config args]
set -o pipefail
tag=${1:-wide}; shift
args=${@:-funnel --dense 0 --warmup 2 --steps 1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pmc_$tag
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/f" -o p -- \
  python3 scripts/bench_configs.py $args > "$O/f.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/w" -o p -- \
  python3 scripts/bench_configs.py $args > "$O/w.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES --output-format csv -d "$O/s" -o p -- \
  python3 scripts/bench_configs.py $args > "$O/s.log" 2>&1 || exit $?
for k in k_wide_v1 k_wide_v2 k_wide_part k_wide_leaf k_wide_rs; do
  echo "== $k"; python3 scripts/pmc_summary.py "$O" "$k"
done > "$O/summary.txt"
rm -rf "$O/f" "$O/w" "$O/s"  # per-dispatch CSVs exceed what gpurun copies back
