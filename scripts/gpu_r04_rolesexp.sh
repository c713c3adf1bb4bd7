# tail form: what bounds its per-tile chain (NMX_ROLES_EXP timing variants, wrong results)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/rx
mkdir -p $O
for r in 1 2; do for v in rx0 rx1 rx2 rx3; do
  echo "== $v"; timeout -k 10 120 python -u scripts/logreg_list_bench.py 1,32,128,256 build/ab/$v/libnumpyro_amd.so 2>&1 | grep -v amdgpu.ids || exit 1
done; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- python3 scripts/logreg_list_bench.py 1,32,256 build/ab/rx0/libnumpyro_amd.so > $O/kt.log 2>&1 || exit 1
python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/kt/*kernel_stats.csv')[0])):
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,2),'us')
" | head -8
rm -f $O/kt/*kernel_trace.csv
