#!/bin/bash
# round 5: the split-bf16 product accuracy guard test
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call42
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -k "x3" -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1; rc=$?
grep -E "x3 accuracy|passed|failed|FAILED" $O/tests.txt | tail -8
exit $rc
