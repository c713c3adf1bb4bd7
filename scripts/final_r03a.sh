#!/bin/bash
# End-of-round-3 GPU check, part A: the whole GPU suite, smoke(), then the step-kernel row-batch A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_steps.sh \
  "tests:420:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "smoke:180:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "abstep:600:bash scripts/ab_step_rows.sh"
rc=$?
cat gpurun_out/steps.log
exit $rc
