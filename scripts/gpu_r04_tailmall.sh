# tail form streaming the compact GEMM1 image (fits the Infinity Cache): tests + A/B vs HEAD
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/tail
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_potentials.py tests/test_gpu_debug_build.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do for v in lgbase lgnew; do
  echo "== $v"; timeout -k 10 120 python -u scripts/logreg_list_bench.py 1,32,64,128,256 build/ab/$v/libnumpyro_amd.so 2>&1 | grep -v amdgpu.ids || exit 1
done; done
for seed in 0 1 2; do for v in lgbase lgnew; do
  timeout -k 10 200 python -u bench.py --chains 512 --configs none --no-cpu-baseline --steps 20 --warmup 5 --seed $seed --lib build/ab/$v/libnumpyro_amd.so > $O/b512_${v}_s$seed.json 2> $O/b512_${v}_s$seed.err || exit 1
  python -c "import json;d=json.load(open('$O/b512_${v}_s$seed.json'));print('$v seed $seed', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3), round(d['roofline']['frac'],4))"
done; done
for v in lgbase lgnew; do
  timeout -k 10 300 python -u bench.py --configs none --no-cpu-baseline --steps 20 --warmup 5 --lib build/ab/$v/libnumpyro_amd.so > $O/b4096_${v}.json 2> $O/b4096_${v}.err || exit 1
  python -c "import json;d=json.load(open('$O/b4096_${v}.json'));print('$v 4096', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3), round(d['roofline']['frac'],4))"
done
