set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/final2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc $?" >> $O/tests.log; tail -3 $O/tests.log
grep -E "FAILED|Error" $O/tests.log | head -20
