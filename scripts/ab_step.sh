# A/B of library builds on the covtype bench: value, mean tree size, launches and per-kernel
# averages (kernel trace).  usage: bash scripts/ab_step.sh "512 4096" "L0A0 L1A1"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for ch in $1; do for v in $2; do
  o=gpurun_out/ab_${v}_${ch}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o k -- python3 bench.py --chains $ch --steps 20 --warmup 5 --no-cpu-baseline --configs none --lib build/ab/$v/libnumpyro_amd.so > $o.json 2>/dev/null || exit 1
  rm -f $o/*kernel_trace.csv
  python3 - "$o" "$ch $v" >> gpurun_out/ab_step.txt <<'PY'
import json, sys, csv, glob
o, tag = sys.argv[1], sys.argv[2]
d = json.loads(open(o + ".json").read().strip().splitlines()[-1])
ks = {}
for r in csv.DictReader(open(glob.glob(o + "/*kernel_stats.csv")[0])):
    n = r["Name"]
    for key in ("k_nuts_step", "k_logreg_finalize", "k_logreg_x3_roles", "k_logreg_x3<"):
        if key in n:
            ks[key] = (int(r["Calls"]), round(float(r["AverageNs"]) / 1e3, 1))
print(tag, round(d["value"]), "tree", round(d["mean_tree_size"], 3), "launches", d.get("launches"), ks)
PY
done; done
