#!/bin/bash
# round 5: stamped narrow tail (experiment build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call12
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u scripts/narrow_stamps.py build/abx/stamps/libnumpyro_amd.so > $O/stamps.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/narrow_stamps.py build/abx/stamps/libnumpyro_amd.so 131072 >> $O/stamps.txt 2>&1 || exit 1
cat $O/stamps.txt
