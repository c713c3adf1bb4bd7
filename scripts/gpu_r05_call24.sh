#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call24
mkdir -p $O
timeout -k 10 300 python -u scripts/step_stamps.py build/abx/stepst/libnumpyro_amd.so 512 20 > $O/step.txt 2>&1 || exit 1
cat $O/step.txt
