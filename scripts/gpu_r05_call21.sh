#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call21
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 scripts/bench_launch_profile.py 512 20 200 5 > $O/launch.txt 2>&1 || exit 1
python3 scripts/kernel_hist.py $O/kt logreg nuts_step > $O/hist.txt || exit 1
rm -rf $O/kt
cat $O/hist.txt
