#!/bin/bash
# round 5: parity suites after the SV double-precision finish, then the full bench line
set -o pipefail
mkdir -p gpurun_out/r05
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_parity_trace.py tests/test_gpu_nuts.py tests/test_gpu_dense.py tests/test_gpu_potentials.py \
  -k "fixed_step or covtype_full or adaptation_matches or trace or bnn_pooled or dense_chain_step_matches_oracle or per_chain_dense_adaptation or structured_dense_mass_matches or dict_of_blocks or sv or stochastic" \
  > gpurun_out/r05/parity_tests2.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r05/parity_tests2.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/r05/bench_call2.json 2> gpurun_out/r05/bench_call2.err
rc=$?
tail -5 gpurun_out/r05/bench_call2.err
exit $rc
