# carry-form leaf rows with HBM-only row batches (NMX_PX_BC): tests, then A/B vs HEAD at SV 8192 / 1024
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/bc
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_debug_build.py tests/test_gpu_parity_trace.py tests/test_gpu_multi_device.py "tests/test_gpu_nuts.py::test_wide_model_step_matches_launched_loop" "tests/test_gpu_nuts.py::test_wide_model_step_invariances" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for C in 8192 1024; do for v in base bc2 bc3 bc4 bc5; do
  timeout -k 10 300 python -u scripts/bench_configs.py sv --chains $C --warmup 100 --steps 10 --lib build/ab/$v/libnumpyro_amd.so > $O/sv_${C}_$v.log 2>&1 || { tail -20 $O/sv_${C}_$v.log; exit 1; }
  echo "C=$C $v $(tail -1 $O/sv_${C}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["leapfrog_per_s"]), d["wall_s"])')"
done; done
