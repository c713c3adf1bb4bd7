#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call16
mkdir -p $O
timeout -k 10 120 python -u scripts/debug_narrow_terms.py build/abx/dbg/libnumpyro_amd.so > $O/dbg.txt 2>&1; cat $O/dbg.txt
