#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call15
mkdir -p $O
timeout -k 10 120 python -u scripts/debug_narrow.py 4001 > $O/dbg.txt 2>&1; cat $O/dbg.txt
