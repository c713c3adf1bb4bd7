#!/bin/bash
# round 5: the dense heuristic-search oracle test with rounding-tie teacher forcing
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call38
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_nuts.py -m gpu -k "heuristic" -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1; rc=$?
grep -E "heuristic dense|PASSED|FAILED|passed|failed" $O/tests.txt | tail -20
exit $rc
