#!/bin/bash
# A/B of the covtype potential's tail form (NMX_X3_TAIL_GT chain tiles or fewer run the
# hand-interleaved kernel) over active-chain counts, one box.  usage: bash scripts/tail_ab.sh
set -o pipefail
mkdir -p gpurun_out
for g in ${SWEEP:-0 2 4 0 2}; do
  echo "tail_gt=$g"
  NMX_X3_TAIL_GT=$g timeout -k 10 120 python -u scripts/logreg_list_bench.py 36 1024,768,512,384,256,128,64,16 || exit 1
done
