set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/occ
mkdir -p $O
timeout -k 10 60 python -u scripts/occ_probe.py build/ab/carry/libnumpyro_amd.so 1000 2000 2519 2530 || exit 1
NMX_PERSIST_CARRY=0 timeout -k 10 60 python -u scripts/occ_probe.py build/ab/carry/libnumpyro_amd.so 2519 || exit 1
for C in 8192 1024; do for v in carry base; do
  timeout -k 10 300 python -u scripts/bench_configs.py sv --chains $C --warmup 100 --steps 10 --lib build/ab/$v/libnumpyro_amd.so > $O/sv_${C}_$v.log 2>&1 || { tail -20 $O/sv_${C}_$v.log; exit 1; }
  echo "C=$C $v"; tail -1 $O/sv_${C}_$v.log | cut -c1-200
done; done
