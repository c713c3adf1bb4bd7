# end-of-round check: full GPU suite, smoke, driver-protocol bench (+ kernel trace of the headline)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc $?" >> $O/tests.log; tail -3 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
