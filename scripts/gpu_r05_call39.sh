#!/bin/bash
# round 5: kernel time split of configs 2 and 3 after the 16x16x32 dense products
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call39
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 scripts/bench_configs.py funnel --chains 4096 --warmup 12 --steps 3 > $O/c2.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- python3 scripts/bench_configs.py bnn --chains 2048 --warmup 20 --steps 2 > $O/c3.log 2>&1 || exit 1
for c in c2 c3; do echo "== $c"; python3 scripts/kernel_hist.py $O/$c | head -12; done > $O/split.txt
find $O -name "*kernel_trace.csv" -delete
cat $O/split.txt | cut -c1-170
