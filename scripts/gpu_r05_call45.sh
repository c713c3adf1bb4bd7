#!/bin/bash
# round 5: the C NUTS restatement's tree-logic loop scheduled dynamic,4 (8 chunks of 32 chains)
# vs dynamic,1 on the box's 16 threads (SV, the c4 CPU leg's shape): leapfrog/s, potential share
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call45
mkdir -p $O
for i in 1 2; do timeout -k 10 120 python3 scripts/sv_cpu_share.py >> $O/dyn4.txt 2>&1 || exit 1; done
sed -i 's/#pragma omp parallel for schedule(dynamic, 4)/#pragma omp parallel for schedule(dynamic, 1)/' oracle/c/nuts_cpu.c
python3 -c "import sys; sys.path.insert(0, '.'); from oracle import build as B; B.build()" || exit 1
for i in 1 2; do timeout -k 10 120 python3 scripts/sv_cpu_share.py >> $O/dyn1.txt 2>&1 || exit 1; done
echo dyn4; cat $O/dyn4.txt; echo dyn1; cat $O/dyn1.txt
