#!/bin/bash
# combined last-k-block A/B: covtype GPU parity tests on HEAD's build, then potential timing
# (HEAD~ vs combined) and bench lines at 512 / 4096 chains.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_steps.sh \
  "ctests:400:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_potentials.py tests/test_gpu_nuts.py tests/test_gpu_debug_build.py" \
  "abcomb:300:AB_REPS=20 AB_ROUNDS=2 python -u scripts/ab_logreg.py build/ab/c2/libnumpyro_amd.so build/ab/comb/libnumpyro_amd.so" \
  "b512:150:python bench.py --chains 512 --configs none --no-cpu-baseline" \
  "b4096:240:python bench.py --configs none --no-cpu-baseline --steps 50"
rc=$?
cat gpurun_out/steps.log; cat gpurun_out/abcomb.log
for f in b512 b4096; do python -c "import json; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],4), round(d['potential_ms_per_launch'],4), round(d['roofline']['frac'],4))"; done
exit $rc
