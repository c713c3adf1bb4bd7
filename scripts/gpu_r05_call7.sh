#!/bin/bash
# round 5: where the covtype potential time goes, by active-chain bucket (4096 and 512 chains)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call7
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/bench_launch_profile.py 4096 20 200 5 > $O/launch_4096.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/bench_launch_profile.py 512 20 200 5 > $O/launch_512.txt 2>&1 || exit 1
cat $O/launch_4096.txt $O/launch_512.txt
