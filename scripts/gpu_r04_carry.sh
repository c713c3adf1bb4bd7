# round 4: LDS-resident frontier of k_wide_persistent -- tests, then A/B (NMX_PERSIST_CARRY=0 vs
# default in the experiment build) at SV 8192 / 1024 chains, then HBM bytes per leapfrog with it
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/carry
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_debug_build.py tests/test_gpu_parity_trace.py tests/test_gpu_multi_device.py "tests/test_gpu_nuts.py::test_wide_model_step_matches_launched_loop" "tests/test_gpu_nuts.py::test_wide_model_step_invariances" "tests/test_gpu_nuts.py::test_persistent_schedule_is_bitwise_the_launched_one" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for C in 8192 1024; do for v in 0 1; do
  NMX_PERSIST_CARRY=$v timeout -k 10 300 python -u scripts/bench_configs.py sv --chains $C --warmup 100 --steps 10 --lib build/ab/carry/libnumpyro_amd.so > $O/sv_${C}_carry$v.log 2>&1 || { tail -20 $O/sv_${C}_carry$v.log; exit 1; }
  echo "C=$C carry=$v"; tail -1 $O/sv_${C}_carry$v.log | cut -c1-400
done; done
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/tf -o p -- python3 scripts/bench_configs.py sv --chains 8192 --warmup 20 --steps 3 > $O/tf.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/tw -o p -- python3 scripts/bench_configs.py sv --chains 8192 --warmup 20 --steps 3 > $O/tw.log 2>&1 || exit 1
mkdir -p $O/traffic/sv && mv $O/tf $O/traffic/sv/f && mv $O/tw $O/traffic/sv/w && cp $O/tf.log $O/traffic/sv/f.log
python3 scripts/traffic_summary.py $O/traffic > $O/traffic_sv.json && rm -rf $O/traffic/sv/f $O/traffic/sv/w
cat $O/traffic_sv.json
