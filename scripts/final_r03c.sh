#!/bin/bash
# End-of-round-3 check on HEAD: the whole GPU suite and smoke().
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_steps.sh \
  "tests:420:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "smoke:180:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
rc=$?
cat gpurun_out/steps.log
exit $rc
