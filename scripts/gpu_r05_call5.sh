#!/bin/bash
# round 5: the whole GPU suite and smoke on the current tree, the SV persistent kernel's VALU
# instruction count (PMC), then the full bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call5
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/gpu_tests.txt 2>&1
rc=$?
tail -3 $O/gpu_tests.txt
grep -E "FAILED|ERROR" $O/gpu_tests.txt | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
tail -1 $O/smoke.txt
