# SQ counters of the persistent SV kernel (carry form), one pass, no trace domains
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/svpmc
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/p1 -o p -- python3 scripts/bench_configs.py sv --chains 8192 --warmup 20 --steps 3 > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d $O/p2 -o p -- python3 scripts/bench_configs.py sv --chains 8192 --warmup 20 --steps 3 > $O/p2.log 2>&1 || exit 1
python3 - << 'PY'
import csv, glob, collections
tot = collections.defaultdict(float)
for f in glob.glob('gpurun_out/svpmc/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_wide_persistent' in r['Kernel_Name']:
            tot[r['Counter_Name']] += float(r['Counter_Value'])
for k, v in sorted(tot.items()):
    print(f"{k:24s} {v:.4g}")
PY
rm -rf gpurun_out/svpmc/p1 gpurun_out/svpmc/p2
