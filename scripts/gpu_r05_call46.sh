#!/bin/bash
# round 5: C NUTS restatement with per-thread chain loops for per-chain potentials (SV probe)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call46
mkdir -p $O
for i in 1 2; do timeout -k 10 120 python3 scripts/sv_cpu_share.py >> $O/perthread.txt 2>&1 || exit 1; done
cat $O/perthread.txt
