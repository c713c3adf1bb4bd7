# end-of-round check after the dense row-layout fusions: dense tests + config profiles, the full
# GPU suite, smoke, and the driver-protocol bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
AB=0 bash scripts/gpu_r04_rowsfuse.sh || exit 1
O=gpurun_out/final4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; echo "tests rc $rc" >> $O/tests.log; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_line.json 2> $O/bench.err || exit 1
tail -c 1500 $O/bench_line.json
