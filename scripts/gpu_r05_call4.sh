#!/bin/bash
# round 5: k_gemm_x3 sweep order A/B (r04 vs chain-block sweep + descending upper triangle):
# timing, bitwise check, HBM bytes (FETCH_SIZE) of the D = 10000 x 4096 product; BNN revert check;
# configs 2-3 with the new product
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/ab4
mkdir -p $O
export PYTHONUNBUFFERED=1
A=build/abx
timeout -k 10 400 python -u scripts/gemm_ab.py $A/gemm_r04/libnumpyro_amd.so $A/gemm_new/libnumpyro_amd.so > $O/gemm.txt 2>&1 || exit 1
cat $O/gemm.txt
for v in gemm_r04 gemm_new; do
  NUMPYRO_AMD_LIB=$A/$v/libnumpyro_amd.so timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/f_$v" -o p -- python3 scripts/bench_gemm_x3.py 10000 4096 5 > $O/f_$v.log 2>&1 || exit 1
  NUMPYRO_AMD_LIB=$A/$v/libnumpyro_amd.so timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/g_$v" -o p -- python3 scripts/bench_gemm_x3.py 5038 2048 5 > $O/g_$v.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, os
O = "gpurun_out/r05/ab4"
for v in ("gemm_r04", "gemm_new"):
    for tag, lab in (("f", "D10000_C4096"), ("g", "D5038_C2048")):
        rows = []
        for f in glob.glob(f"{O}/{tag}_{v}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_gemm_x3" in r.get("Kernel_Name", ""):
                    rows.append(float(r["Counter_Value"]))
        if rows:
            print(v, lab, "FETCH_SIZE per dispatch (KB, x2 gfx950 correction -> GB):", len(rows), round(sum(rows) / len(rows) * 2 * 1024 / 1e9, 3), "GB")
PY
timeout -k 10 300 python -u scripts/ab_bnn.py $A/bnn_r04/libnumpyro_amd.so $A/bnn_rev/libnumpyro_amd.so > $O/bnn.txt 2>&1 || exit 1
cat $O/bnn.txt
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --adapt 30 --no-cpu-baseline --configs c2,c3 > $O/cfg.json 2> $O/cfg.err || exit 1
python3 -c "import json;d=json.load(open('$O/cfg.json'));[print(k, round(v['value']), round(v['roofline']['frac'],4), v['roofline'].get('potential_launches',{}).get('frac')) for k,v in d['configs'].items()]"
