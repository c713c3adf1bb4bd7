#!/bin/bash
# round 5: narrow tail v3 (three-stage pipeline): bitwise tests, list timings, stamps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call31
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_potentials.py -k "logreg" > $O/tests.txt 2>&1
rc=$?
tail -2 $O/tests.txt
grep -E "FAILED|ERROR|Error" $O/tests.txt | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/logreg_list_bench.py 1,16,32,33 > $O/list.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/narrow_stamps.py build/abx/stamps/libnumpyro_amd.so > $O/stamps.txt 2>&1 || exit 1
cat $O/list.txt $O/stamps.txt
