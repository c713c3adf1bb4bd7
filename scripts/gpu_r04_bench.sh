# round-4 bench call: the driver's command line (bench.py --steps 20 --warmup 5), then the
# headline under rocprofv3 kernel-trace + stats (timed-launch averages vs the in-run roofline)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_line.json 2> $O/bench.err || exit 1
tail -c 600 $O/bench_line.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o b -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --configs none > $O/kt_line.json 2> $O/kt.err || exit 1
python3 scripts/trace_timed_avg.py $(ls $O/kt/*kernel_trace.csv | head -1) $O/kt_line.json > $O/bench_timed_kernel_avg.json || exit 1
rm -f $O/kt/*kernel_trace.csv
cat $O/bench_timed_kernel_avg.json
