#!/bin/bash
# Round profiling on the GPU box: bench line, rocprofv3 kernel stats of bench.py, PMC HBM
# traffic of the dominant kernel (FETCH_SIZE / WRITE_SIZE in separate passes, per
# MI355X_MICROARCH.md), and the secondary-config benches.  Stops at the first failure.
# usage: bash scripts/profile_round.sh <tag>      -> gpurun_out/prof_<tag>/
set -o pipefail
tag=${1:-r01}
part=${2:-all}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/prof_$tag
mkdir -p "$O"
step() { echo "== $1" >> "$O/steps.log"; shift; "$@"; rc=$?; echo "rc=$rc" >> "$O/steps.log"; [ $rc -eq 0 ] || exit $rc; }
if [ "$part" != b ]; then
step fetch timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o p -- python3 scripts/bench_potential.py d 4096
step write timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o p -- python3 scripts/bench_potential.py d 4096
step traffic python3 scripts/traffic_json.py "$O/pmc_fetch" "$O/pmc_write" "$O/traffic.json" "k_logreg_x3, C=4096 all active"
# the bench line reports this round's PMC traffic (bench.py --traffic-json)
step bench timeout -k 10 600 bash -c "python bench.py --traffic-json $O/traffic.json > $O/bench_line.json 2> $O/bench.err"
step ktrace timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrace" -o bench -- python3 bench.py --no-cpu-baseline --traffic-json $O/traffic.json
step timedavg bash -c "python3 scripts/trace_timed_avg.py \$(ls $O/ktrace/*kernel_trace.csv | head -1) $O/bench_line.json > $O/bench_timed_kernel_avg.json"
step sqpmc bash scripts/pmc_kernel.sh d "$tag"
fi
[ "$part" = a ] && { echo done >> "$O/steps.log"; exit 0; }
step configs timeout -k 10 900 bash -c "python scripts/bench_configs.py gemm 10000 4096 > $O/configs.jsonl && \
  python scripts/bench_configs.py covtype --chains 1024 --warmup 30 --steps 10 >> $O/configs.jsonl && \
  python scripts/bench_configs.py funnel --dense 0 --warmup 10 --steps 3 >> $O/configs.jsonl && \
  python scripts/bench_configs.py funnel --warmup 10 --steps 2 >> $O/configs.jsonl && \
  python scripts/bench_configs.py bnn --warmup 10 --steps 3 >> $O/configs.jsonl && \
  python scripts/bench_configs.py sv --chains 1024 --warmup 10 --steps 3 >> $O/configs.jsonl && \
  python scripts/bench_configs.py sv --chains 8192 --warmup 10 --steps 3 >> $O/configs.jsonl"
step fprof timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrace_funnel_dense" -o f -- python3 scripts/bench_configs.py funnel --warmup 10 --steps 2
echo done >> "$O/steps.log"
