#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call28
mkdir -p $O
timeout -k 10 400 python -u scripts/debug_pooled_determinism.py > $O/det.txt 2>&1 || exit 1
cat $O/det.txt
