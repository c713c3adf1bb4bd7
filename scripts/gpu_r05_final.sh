#!/bin/bash
# round 5 end-of-round check: full GPU suite, smoke, in-run HBM traffic (separate FETCH/WRITE
# passes), the default bench line with that traffic record, and the headline's kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
echo "tests rc $rc" >> $O/tests.log; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
