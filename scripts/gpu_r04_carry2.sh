# round 4: persistent kernel with frontier + inverse mass in LDS: tests, A/B vs arena, phase profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/carry2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_debug_build.py tests/test_gpu_parity_trace.py tests/test_gpu_multi_device.py "tests/test_gpu_nuts.py::test_wide_model_step_matches_launched_loop" "tests/test_gpu_nuts.py::test_wide_model_step_invariances" "tests/test_gpu_nuts.py::test_persistent_schedule_is_bitwise_the_launched_one" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for C in 8192 1024; do for v in 0 1; do
  NMX_PERSIST_CARRY=$v timeout -k 10 300 python -u scripts/bench_configs.py sv --chains $C --warmup 100 --steps 10 --lib build/ab/carry/libnumpyro_amd.so > $O/sv_${C}_carry$v.log 2>&1 || { tail -20 $O/sv_${C}_carry$v.log; exit 1; }
  echo "C=$C carry=$v"; tail -1 $O/sv_${C}_carry$v.log | cut -c1-200
done; done
for C in 8192 1024; do
  timeout -k 10 200 python -u scripts/px_profile.py sv $C > $O/px_sv_$C.log 2>&1 || { tail -20 $O/px_sv_$C.log; exit 1; }
  grep -v amdgpu.ids $O/px_sv_$C.log
done
