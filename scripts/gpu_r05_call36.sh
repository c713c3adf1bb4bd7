#!/bin/bash
# round 5: k_gemm_x3 with A staged as f32 and split in registers (4 instead of 6 B of A per
# value): A/B against the pre-split build (bitwise equal products expected), dense GPU tests,
# c2 / c3 bench legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call36
mkdir -p $O
timeout -k 10 300 python3 -u scripts/gemm_ab.py build/abx/gemm_b16a/libnumpyro_amd.so numpyro_amd/_lib/libnumpyro_amd.so build/abx/gemm_b16a/libnumpyro_amd.so numpyro_amd/_lib/libnumpyro_amd.so > $O/gemm_ab.txt 2>&1 || { tail -20 $O/gemm_ab.txt; exit 1; }
grep RESULT $O/gemm_ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --configs c2,c3 --no-cpu-baseline > $O/bench_c23.json 2> $O/bench_c23.err || exit 1
python3 -c "
import json
d=json.loads(open('$O/bench_c23.json').readline())
for k in ('c2','c3'):
    c=d['configs'][k]
    print(k, round(c['value']), round(c['roofline']['frac'],4))"
