#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call26
mkdir -p $O
timeout -k 10 120 python -u scripts/fin_stamps.py build/abx/finst/libnumpyro_amd.so 1 > $O/fin.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/fin_stamps.py build/abx/finst/libnumpyro_amd.so 32 >> $O/fin.txt 2>&1 || exit 1
cat $O/fin.txt
