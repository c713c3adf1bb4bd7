#!/bin/bash
# round 5: step-kernel reduction: covtype GPU tests (bitwise-sensitive), stamps, launch profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call20
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.txt 2>&1
rc=$?
tail -2 $O/tests.txt
grep -E "FAILED|ERROR" $O/tests.txt | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/step_stamps.py build/abx/stepst/libnumpyro_amd.so 512 20 > $O/step.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/bench_launch_profile.py 512 20 200 5 > $O/launch_512.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/bench_launch_profile.py 4096 20 200 5 > $O/launch_4096.txt 2>&1 || exit 1
cat $O/step.txt $O/launch_512.txt $O/launch_4096.txt
