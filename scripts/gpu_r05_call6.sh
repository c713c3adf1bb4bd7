#!/bin/bash
# round 5: dense + find_heuristic_step_size and pooled structured mass on the GPU, then the SV
# persistent kernel's VALU counters with its kernel trace (one PMC pass, no trace domains)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call6
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dense.py tests/test_gpu_nuts.py -k "heuristic or dense or pooled" > $O/tests.txt 2>&1
rc=$?
tail -3 $O/tests.txt
grep -E "FAILED|ERROR" $O/tests.txt | head
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --stats --output-format csv -d $O/pmc -o p -- python3 scripts/bench_configs.py sv --chains 8192 --warmup 20 --steps 3 > $O/sv_pmc.log 2>&1 || exit 1
python3 scripts/valu_summary.py $O/pmc $O/sv_pmc.log k_wide_persistent > $O/sv_valu.txt || exit 1
cat $O/sv_valu.txt
rm -rf $O/pmc
