#!/bin/bash
# round 5: k_gemm_x3 on 16x16x32 sub-tiles vs 32x32x16 (same staged pieces, same products per
# output, different MFMA shape): A/B timing, product accuracy, dense GPU tests, c2 / c3 legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call37
mkdir -p $O
timeout -k 10 300 python3 -u scripts/gemm_ab.py build/abx/gemm_32/libnumpyro_amd.so numpyro_amd/_lib/libnumpyro_amd.so > $O/gemm_ab.txt 2>&1 || { tail -20 $O/gemm_ab.txt; exit 1; }
grep RESULT $O/gemm_ab.txt
timeout -k 10 300 python3 -u scripts/gemm_ab.py numpyro_amd/_lib/libnumpyro_amd.so build/abx/gemm_32/libnumpyro_amd.so > $O/gemm_ab2.txt 2>&1 || { tail -20 $O/gemm_ab2.txt; exit 1; }
grep RESULT $O/gemm_ab2.txt
timeout -k 10 300 python3 -u scripts/bnn_accuracy.py 64 > $O/bnn_accuracy.txt 2>&1 || { tail -20 $O/bnn_accuracy.txt; exit 1; }
grep -A4 gemm_device $O/bnn_accuracy.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --configs c2,c3 --no-cpu-baseline > $O/bench_c23.json 2> $O/bench_c23.err || exit 1
python3 -c "
import json
d=json.loads(open('$O/bench_c23.json').readline())
for k in ('c2','c3'):
    c=d['configs'][k]
    print(k, round(c['value']), round(c['roofline']['frac'],4))"
