#!/bin/bash
# HBM bytes per dispatch (rocprofv3 FETCH_SIZE and WRITE_SIZE, one counter per pass, no trace
# domains) of the kernels the bench rooflines rest on:
#   k_logreg_x3 (+ finalize)     scripts/bench_potential.py d 4096   (all 4096 covtype chains active)
#   k_wide_persistent (SV)       scripts/bench_configs.py sv --chains 8192 --warmup 20 --steps 3
#   k_gemm_x3 <4,2,8>            scripts/bench_gemm_x3.py 10000 4096 (upper triangle, all active)
#   k_chain_step, k_gemm_x3      scripts/bench_configs.py funnel --chains 4096 --warmup 12 --steps 2 (dense pooled)
# -> gpurun_out/traffic/<workload>/{f,w}/ ; summarized by scripts/traffic_summary.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/traffic
mkdir -p "$O"
run() {  # name, command...
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/$n/f" -o p -- "$@" > "$O/$n/f.log" 2>&1 || return $?
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/$n/w" -o p -- "$@" > "$O/$n/w.log" 2>&1 || return $?
}
mkdir -p $O/logreg $O/sv $O/gemm $O/funnel
run logreg python3 scripts/bench_potential.py d 4096 || exit 1
run sv python3 scripts/bench_configs.py sv --chains 8192 --warmup 20 --steps 3 || exit 1
run gemm python3 scripts/bench_gemm_x3.py 10000 4096 5 || exit 1
run funnel python3 scripts/bench_configs.py funnel --chains 4096 --warmup 12 --steps 2 || exit 1
python3 scripts/traffic_summary.py "$O" > "$O/summary.json" || exit 1
for n in logreg sv gemm funnel; do rm -rf "$O/$n/f" "$O/$n/w"; done
cat "$O/summary.json"
