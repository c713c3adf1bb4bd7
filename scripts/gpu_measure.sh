#!/bin/bash
# end-of-round measurement (usage: bash scripts/gpu_measure.sh [OUT_DIR]): in-run HBM traffic of the headline (FETCH_SIZE and
# WRITE_SIZE in separate passes), the default bench line, and the headline's rocprof kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/measure}
mkdir -p $O/t
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/t/f -o p -- python3 bench.py --steps 20 --warmup 5 --configs none --no-cpu-baseline > $O/t/f.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/t/w -o p -- python3 bench.py --steps 20 --warmup 5 --configs none --no-cpu-baseline > $O/t/w.log 2>&1 || exit 1
python3 scripts/bench_traffic_summary.py $O/t > $O/traffic.json || exit 1
rm -rf $O/t/f $O/t/w
cat $O/traffic.json | cut -c1-400
timeout -k 10 1100 python -u bench.py --traffic-json $O/traffic.json > $O/bench.json 2> $O/bench.err || exit 1
head -c 600 $O/bench.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --configs none --no-cpu-baseline --traffic-json $O/traffic.json > $O/prof.log 2>&1 || exit 1
python3 scripts/kernel_hist.py $O/prof > $O/headline_kernel_hist.txt && cat $O/headline_kernel_hist.txt
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/headline_kernel_stats.csv \;
python3 scripts/bench_timed_kernel_avg.py $O/prof $O/prof.log > $O/timed_kernel_avg.json && cat $O/timed_kernel_avg.json
