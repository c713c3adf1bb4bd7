#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call22
mkdir -p $O
timeout -k 10 60 ./scripts/micro/launch_floor > $O/floor.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- ./scripts/micro/launch_floor > $O/floor_prof.txt 2>&1 || exit 1
python3 scripts/kernel_hist.py $O/kt like >> $O/floor.txt || exit 1
rm -rf $O/kt
cat $O/floor.txt
