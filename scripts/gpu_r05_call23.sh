#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call23
mkdir -p $O
timeout -k 10 200 python -u scripts/step_floor.py 512 > $O/floor.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/step_floor.py 4096 >> $O/floor.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 scripts/step_floor.py 512 > $O/prof.txt 2>&1 || exit 1
python3 scripts/kernel_hist.py $O/kt nuts_step >> $O/floor.txt || exit 1
rm -rf $O/kt
cat $O/floor.txt
