# rocprof kernel stats of the config workloads on the final round-4 HEAD
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/cfgprof
mkdir -p $O
for w in "sv --chains 8192 --warmup 50 --steps 5" "bnn --chains 2048 --warmup 20 --steps 2" "funnel --chains 4096 --warmup 12 --steps 2"; do
  n=$(echo $w | cut -d' ' -f1)
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o k -- python3 scripts/bench_configs.py $w > $O/$n.log 2>&1 || exit 1
  rm -f $O/$n/*kernel_trace.csv
  python3 -c "
import csv,glob
rows=list(csv.DictReader(open(glob.glob('$O/$n/*kernel_stats.csv')[0])))
print('== $n')
for r in rows[:8]: print(f\"{r['Name'][:78]:78s} {int(r['Calls']):7d} {float(r['TotalDurationNs'])/1e6:9.1f} ms {float(r['AverageNs'])/1e3:9.2f} us {float(r['Percentage']):5.1f}%\")
"
done
