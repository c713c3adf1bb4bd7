#!/bin/bash
# round 5: tail potential time vs rows (X resident in the Infinity Cache or not), kernel split
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call11
mkdir -p $O
export PYTHONUNBUFFERED=1
for N in 65536 131072 262144 581012 1162024; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt$N -o kt -- python3 scripts/tail_rows_bench.py $N 1 > $O/n$N.log 2>&1 || exit 1
  grep "^N " $O/n$N.log >> $O/rows.txt
  python3 scripts/kernel_hist.py $O/kt$N roles finalize >> $O/rows.txt || exit 1
  rm -rf $O/kt$N
done
cat $O/rows.txt
