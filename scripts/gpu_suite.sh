#!/bin/bash
# end-of-round check (usage: bash scripts/gpu_suite.sh [OUT_DIR]): full GPU suite, smoke, in-run HBM traffic (separate FETCH/WRITE
# passes), the default bench line with that traffic record, and the headline's kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-gpurun_out/suite}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
echo "tests rc $rc" >> $O/tests.log; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
# the driver's multi-GPU bench command rehearsed with 2 ranks on the one GPU (gloo collectives;
# the driver's own runs use RCCL, one rank per GPU)
NMX_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 > $O/rehearsal_n2.json 2> $O/rehearsal_n2.err || { tail -20 $O/rehearsal_n2.err; exit 1; }
head -c 700 $O/rehearsal_n2.json; echo
