# Fused row-gather split of the dense products (nmx_gemm_chains_x3_rows) vs nmx_pack_rows + split:
# dense GPU tests, then configs 2 (funnel-10k dense) and 3 (BNN dense) A/B under rocprof stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/rowsfuse
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dense.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for ab in ${AB:-0 1}; do
for w in "bnn --chains 2048 --warmup 20 --steps 2" "funnel --chains 4096 --warmup 12 --steps 2"; do
  n=$(echo $w | cut -d' ' -f1)_$ab
  NMX_DENSE_PACK_ROWS=$ab timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o k -- python3 scripts/bench_configs.py $w > $O/$n.log 2>&1 || exit 1
  rm -f $O/$n/*kernel_trace.csv
  tail -1 $O/$n.log
  python3 -c "
import csv,glob
rows=list(csv.DictReader(open(glob.glob('$O/$n/*kernel_stats.csv')[0])))
print('== $n', 'total %.1f ms' % (sum(float(r['TotalDurationNs']) for r in rows)/1e6))
for r in rows[:8]: print(f\"{r['Name'][:78]:78s} {int(r['Calls']):7d} {float(r['TotalDurationNs'])/1e6:9.1f} ms {float(r['AverageNs'])/1e3:9.2f} us {float(r['Percentage']):5.1f}%\")
"
done
done
