#!/bin/bash
# round 5: config 4 (SV, 8192 chains) in a converged regime: the reference example's 1000
# adaptation transitions, 200 timed draws (split R-hat over 200 draws per chain)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call34
mkdir -p $O
timeout -k 10 300 python3 -u scripts/bnn_accuracy.py 64 > $O/bnn_accuracy.txt 2>&1 || { tail -20 $O/bnn_accuracy.txt; exit 1; }
cat $O/bnn_accuracy.txt
timeout -k 10 900 python3 -u scripts/bench_configs.py sv --chains 8192 --warmup 1000 --steps 200 > $O/sv8192_W1000_S200.txt 2>&1 || { tail -20 $O/sv8192_W1000_S200.txt; exit 1; }
grep '^{' $O/sv8192_W1000_S200.txt
