#!/bin/bash
# round 5: config 2 (funnel D=10000, 4096 chains, dense pooled) over 100 timed draws after the
# bench's W=100 adaptation: split R-hat over 100 draws per chain instead of 5
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call43
mkdir -p $O
timeout -k 10 900 python3 -u scripts/bench_configs.py funnel --chains 4096 --warmup 100 --steps 100 > $O/c2_W100_S100.txt 2>&1 || { tail -20 $O/c2_W100_S100.txt; exit 1; }
grep '^{' $O/c2_W100_S100.txt
