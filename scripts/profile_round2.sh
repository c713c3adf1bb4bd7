#!/bin/bash
# Round-2 refresh on the GPU box: the driver-protocol bench line (configs included), a kernel
# trace of the headline run (stats + timed-launch averages), the timeline of one rank's share at
# 8 GPUs (512 chains), and kernel stats of the SV config's per-rank share.  -> gpurun_out/r02b/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02b
mkdir -p "$O"
step() { echo "== $1" >> "$O/steps.log"; shift; "$@"; rc=$?; echo "rc=$rc" >> "$O/steps.log"; [ $rc -eq 0 ] || exit $rc; }
step bench timeout -k 10 500 bash -c "python bench.py --steps 20 --warmup 5 > $O/bench_line.json 2> $O/bench.err"
step ktrace timeout -k 10 300 bash -c "rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o b -- python3 bench.py --no-cpu-baseline --configs none > $O/kt_line.json 2> $O/kt.err"
step timedavg bash -c "python3 scripts/trace_timed_avg.py \$(ls $O/kt/*kernel_trace.csv | head -1) $O/kt_line.json > $O/bench_timed_kernel_avg.json && python3 scripts/trace_timeline.py \$(ls $O/kt/*kernel_trace.csv | head -1) $O/kt_line.json > $O/timeline_4096.json && rm -f $O/kt/*kernel_trace.csv"
step t512 timeout -k 10 300 bash -c "rocprofv3 --kernel-trace --output-format csv -d $O/t512 -o t -- python3 bench.py --chains 512 --no-cpu-baseline --configs none > $O/b512_line.json 2> $O/b512.err"
step tl512 bash -c "python3 scripts/trace_timeline.py \$(ls $O/t512/*kernel_trace.csv | head -1) $O/b512_line.json > $O/timeline_rank512.json && rm -rf $O/t512"
step sv timeout -k 10 300 bash -c "rocprofv3 --kernel-trace --stats --output-format csv -d $O/sv -o s -- python3 scripts/bench_configs.py sv --chains 1024 --warmup 50 --steps 20 > $O/sv_line.json 2> $O/sv.err && rm -f $O/sv/*kernel_trace.csv"
echo done >> "$O/steps.log"
