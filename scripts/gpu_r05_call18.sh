#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call18
mkdir -p $O
rm -f $O/stamps.txt
for v in stamps nomma noload; do
  echo "== $v" >> $O/stamps.txt
  timeout -k 10 120 python -u scripts/narrow_stamps.py build/abx/$v/libnumpyro_amd.so > $O/$v.txt 2>&1 || exit 1
  sed -n 2,7p $O/$v.txt >> $O/stamps.txt
done
cat $O/stamps.txt
