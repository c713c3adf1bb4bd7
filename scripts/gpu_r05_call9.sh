#!/bin/bash
# round 5: narrow tail form (<= 32 listed chains): bitwise tests, list timings, launch profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call9
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_potentials.py -k "logreg" > $O/tests.txt 2>&1
rc=$?
tail -3 $O/tests.txt
grep -E "FAILED|ERROR|Error" $O/tests.txt | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/logreg_list_bench.py 1,16,32,33,64,128,256 > $O/list.txt 2>&1 || exit 1
cat $O/list.txt
timeout -k 10 300 python -u scripts/bench_launch_profile.py 512 20 200 5 > $O/launch_512.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/bench_launch_profile.py 4096 20 200 5 > $O/launch_4096.txt 2>&1 || exit 1
cat $O/launch_512.txt $O/launch_4096.txt
