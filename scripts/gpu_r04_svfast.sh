# SV row math experiment (NMX_SV_FAST: hardware rcp / log2 forms): A/B at 8192 / 1024 chains
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/svfast
mkdir -p $O
for C in 8192 1024; do for v in svbase svfast; do
  timeout -k 10 300 python -u scripts/bench_configs.py sv --chains $C --warmup 100 --steps 10 --lib build/ab/$v/libnumpyro_amd.so > $O/sv_${C}_$v.log 2>&1 || { tail -20 $O/sv_${C}_$v.log; exit 1; }
  echo "C=$C $v $(tail -1 $O/sv_${C}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["leapfrog_per_s"]), d["wall_s"], d["mean_tree"], d["leapfrogs"])')"
done; done
