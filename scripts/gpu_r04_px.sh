# persistent wide kernel with the LDS frontier: per-phase cycles (NMX_PX_PROF build) and the
# leaf-phase row batch A/B (NMX_PX_BL 2 vs 3) at SV 8192 / 1024 chains
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/px
mkdir -p $O
for C in 8192 1024; do
  timeout -k 10 200 python -u scripts/px_profile.py sv $C > $O/px_sv_$C.log 2>&1 || { tail -20 $O/px_sv_$C.log; exit 1; }
  cat $O/px_sv_$C.log | grep -v amdgpu.ids
done
for C in 8192 1024; do for v in carry bl3; do
  timeout -k 10 300 python -u scripts/bench_configs.py sv --chains $C --warmup 100 --steps 10 --lib build/ab/$v/libnumpyro_amd.so > $O/sv_${C}_$v.log 2>&1 || { tail -20 $O/sv_${C}_$v.log; exit 1; }
  echo "C=$C $v"; tail -1 $O/sv_${C}_$v.log | cut -c1-200
done; done
