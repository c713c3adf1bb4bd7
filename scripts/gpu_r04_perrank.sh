# one rank's share at 8 GPUs on the final HEAD: covtype 512 chains (seeds 0-2), SV 1024 chains
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/perrank
mkdir -p $O
for seed in 0 1 2; do
  timeout -k 10 200 python -u bench.py --chains 512 --configs none --no-cpu-baseline --steps 20 --warmup 5 --seed $seed > $O/b512_s$seed.json 2> $O/b512_s$seed.err || exit 1
  python3 -c "import json;d=json.load(open('$O/b512_s$seed.json'));print('covtype 512 seed $seed', round(d['value']), d['leapfrog_launches'], round(d['ms_per_step'],3), round(d['roofline']['frac'],4))"
done
timeout -k 10 300 python -u scripts/bench_configs.py sv --chains 1024 --warmup 200 --steps 10 > $O/sv1024.log 2>&1 || exit 1
echo "SV 1024 $(tail -1 $O/sv1024.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["leapfrog_per_s"]), d["wall_s"], d["mean_tree"])')"
