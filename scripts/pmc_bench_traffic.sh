#!/bin/bash
# HBM bytes per potential launch INSIDE the bench's timed region (the roofline's `traffic`):
# rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over the headline bench run
# (no configs, no CPU baseline); scripts/bench_traffic_summary.py averages k_logreg_x3 (main or
# tail form) + k_logreg_finalize over the last `leapfrog_launches` dispatches (the timed ones).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/traffic_bench
mkdir -p "$O"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/f" -o p -- python3 bench.py --steps 20 --warmup 5 --configs none --no-cpu-baseline > "$O/f.log" 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/w" -o p -- python3 bench.py --steps 20 --warmup 5 --configs none --no-cpu-baseline > "$O/w.log" 2>&1 || exit 1
python3 scripts/bench_traffic_summary.py "$O" > "$O/summary.json" || exit 1
rm -rf "$O/f" "$O/w"
cat "$O/summary.json"
