#!/bin/bash
# round 5: kernel-duration histograms of the covtype run at 512 and 4096 chains (kernel trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call8
mkdir -p $O
export PYTHONUNBUFFERED=1
for C in 512 4096; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt$C -o kt -- python3 scripts/bench_launch_profile.py $C 20 200 5 > $O/launch_$C.txt 2>&1 || exit 1
  python3 scripts/kernel_hist.py $O/kt$C logreg nuts_step > $O/hist_$C.txt || exit 1
  rm -rf $O/kt$C
done
cat $O/hist_512.txt $O/hist_4096.txt
