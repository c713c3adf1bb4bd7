#!/bin/bash
# round 5: the headline's rocprof kernel trace + stats (csv) and the timed-launch average of the
# potential kernels against the bench line's in-run HIP-event figure
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/final_prof
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --configs none --no-cpu-baseline --traffic-json gpurun_out/r05/final_bench/traffic.json > $O/prof.log 2>&1 || exit 1
python3 scripts/kernel_hist.py $O/prof > $O/headline_kernel_hist.txt && cat $O/headline_kernel_hist.txt
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/headline_kernel_stats.csv \;
python3 scripts/bench_timed_kernel_avg.py $O/prof $O/prof.log > $O/timed_kernel_avg.json && cat $O/timed_kernel_avg.json
find $O/prof -name "*kernel_trace.csv" -delete
