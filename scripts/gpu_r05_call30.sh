#!/bin/bash
# round 5: narrow tail form with wave priorities (A/B waves over the DMA / split helpers)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call30
mkdir -p $O
rm -f $O/list.txt
for v in base prio prio2 base prio prio2; do
  L=build/abx/$v/libnumpyro_amd.so; [ $v = base ] && L=numpyro_amd/_lib/libnumpyro_amd.so
  echo "== $v" >> $O/list.txt
  timeout -k 10 200 python -u scripts/logreg_list_bench.py 1,16,32 $L >> $O/list.txt 2>&1 || exit 1
done
cat $O/list.txt
