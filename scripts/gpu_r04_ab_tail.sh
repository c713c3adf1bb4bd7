# A/B of the roles tail kernel's prefetch depth (NMX_X3_ROLE_PA): potential launch time over
# compacted lists, then bench.py --chains 512 (one rank's share at 8 GPUs), seeds 0-2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in pa2 pa4 pa6; do
  echo "== $v"; timeout -k 10 120 python -u scripts/logreg_list_bench.py 1,32,64,128,256,257,512 build/ab/$v/libnumpyro_amd.so || exit 1
done
for seed in 0 1 2; do for v in pa2 pa4; do
  timeout -k 10 200 python -u bench.py --chains 512 --configs none --no-cpu-baseline --steps 20 --warmup 5 --seed $seed --lib build/ab/$v/libnumpyro_amd.so > gpurun_out/b512_${v}_s$seed.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b512_${v}_s$seed.json'));print('$v seed $seed', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3), round(d['roofline']['frac'],4))"
done; done
