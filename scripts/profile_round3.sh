#!/bin/bash
# Round-3 profiles on the GPU box -> gpurun_out/r03/: rocprofv3 kernel stats of the BASELINE
# configs 2 (funnel-10k dense), 3 (BNN dense) and 4 (SV 8192, persistent) in their bench regimes, and of the headline
# run (timed-launch averages for the roofline cross-check).  Traces are reduced and deleted.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03
mkdir -p "$O"
step() { echo "== $1" >> "$O/steps.log"; shift; "$@"; rc=$?; echo "rc=$rc" >> "$O/steps.log"; [ $rc -eq 0 ] || exit $rc; }
W2=${W2:-100}
W3=${W3:-100}
what=${1:-all}
if [ "$what" = all ] || [ "$what" = c2 ]; then
step c2 timeout -k 10 500 bash -c "rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o c2 -- python3 scripts/bench_configs.py funnel --dim 10000 --chains 4096 --warmup $W2 --steps 5 > $O/c2_line.json 2> $O/c2.err; rc=\$?; rm -f $O/c2/*kernel_trace.csv; exit \$rc"
fi
if [ "$what" = all ] || [ "$what" = c3 ]; then
step c3 timeout -k 10 400 bash -c "rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o c3 -- python3 scripts/bench_configs.py bnn --chains 2048 --warmup $W3 --steps 5 > $O/c3_line.json 2> $O/c3.err; rc=\$?; rm -f $O/c3/*kernel_trace.csv; exit \$rc"
fi
if [ "$what" = all ] || [ "$what" = c4 ]; then
step c4 timeout -k 10 300 bash -c "rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o c4 -- python3 scripts/bench_configs.py sv --chains 8192 --warmup 200 --steps 10 > $O/c4_line.json 2> $O/c4.err; rc=\$?; rm -f $O/c4/*kernel_trace.csv; exit \$rc"
fi
if [ "$what" = all ] || [ "$what" = head ]; then
step ktrace timeout -k 10 300 bash -c "rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o b -- python3 bench.py --no-cpu-baseline --configs none > $O/kt_line.json 2> $O/kt.err"
step timedavg bash -c "python3 scripts/trace_timed_avg.py \$(ls $O/kt/*kernel_trace.csv | head -1) $O/kt_line.json > $O/bench_timed_kernel_avg.json && rm -f $O/kt/*kernel_trace.csv"
fi
echo done >> "$O/steps.log"
