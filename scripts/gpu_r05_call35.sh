#!/bin/bash
# round 5: k_gemm_x3 with the correction products in a second accumulator: A/B timing against
# the previous build, product accuracy at D = 5038, dense GPU tests, c2 / c3 bench legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call35
mkdir -p $O
timeout -k 10 300 python3 -u scripts/gemm_ab.py build/abx/gemm_old/libnumpyro_amd.so numpyro_amd/_lib/libnumpyro_amd.so > $O/gemm_ab.txt 2>&1 || { tail -20 $O/gemm_ab.txt; exit 1; }
grep RESULT $O/gemm_ab.txt
timeout -k 10 300 python3 -u scripts/bnn_accuracy.py 64 > $O/bnn_accuracy.txt 2>&1 || { tail -20 $O/bnn_accuracy.txt; exit 1; }
grep -A4 gemm_ $O/bnn_accuracy.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_parity_trace.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --configs c2,c3 > $O/bench_c23.json 2> $O/bench_c23.err || exit 1
python3 -c "
import json
d=json.loads(open('$O/bench_c23.json').readline())
for k in ('c2','c3'):
    c=d['configs'][k]; p=c['parity']
    print(k, round(c['value']), round(c['roofline']['frac'],4), {x:p.get(x) for x in ('matched','unexplained')}, p['draw_drift'].get('geo_mean_ratio'), p['draw_drift'].get('geo_mean_lo95'), p['calibration']['device_like_calibration'])"
grep -E "rounding drift|NOT explained" $O/bench_c23.err | grep -v "no rounding calibration" | cut -c1-300
