#!/bin/bash
# End-of-round-3 GPU check, part B: the default bench line (headline + configs 2-4), then the
# headline's rocprofv3 kernel stats with the timed-launch average cross-check (profile_round3.sh head).
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_steps.sh "bench:660:python -u bench.py > gpurun_out/bench_line.json" || { cat gpurun_out/steps.log; exit 1; }
tail -c 600 gpurun_out/bench_line.json
O=gpurun_out/r03 bash scripts/profile_round3.sh head
rc=$?
cat gpurun_out/steps.log gpurun_out/r03/steps.log 2>/dev/null
exit $rc
