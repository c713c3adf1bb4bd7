#!/bin/bash
# round 5: narrow tail prefetch depth A/B (list timings incl. finalize) + kernel trace split
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call10
mkdir -p $O
export PYTHONUNBUFFERED=1
for v in pf1 main pf3 pf1 main pf3; do
  L=build/abx/$v/libnumpyro_amd.so; [ $v = main ] && L=numpyro_amd/_lib/libnumpyro_amd.so
  echo "== $v" >> $O/list.txt
  timeout -k 10 200 python -u scripts/logreg_list_bench.py 1,16,32 $L >> $O/list.txt 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 scripts/logreg_list_bench.py 1,32,64 > $O/kt.log 2>&1 || exit 1
python3 scripts/kernel_hist.py $O/kt logreg > $O/hist.txt || exit 1
rm -rf $O/kt
cat $O/list.txt $O/hist.txt
