#!/bin/bash
# round 5: leaf-located parity suites (bounded draws, float64 references) on the GPU
set -o pipefail
mkdir -p gpurun_out/r05
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_parity_trace.py tests/test_gpu_nuts.py tests/test_gpu_dense.py \
  -k "fixed_step or covtype_full or adaptation_matches or trace or bnn_pooled or dense_chain_step_matches_oracle or per_chain_dense_adaptation or structured_dense_mass_matches or dict_of_blocks" \
  > gpurun_out/r05/parity_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r05/parity_tests.log | tail -60
exit $rc
