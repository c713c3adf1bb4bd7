cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pbnn -o b -- python3 scripts/bench_bnn.py 69 > gpurun_out/pbnn.log 2>&1 || exit 1
rm -f gpurun_out/pbnn/*kernel_trace.csv
