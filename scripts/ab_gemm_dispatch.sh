#!/bin/bash
# Dense configs with the tile dispatch of nmx_gemm_chains_x3 (default library) vs 128 x 64 tiles
# always (build/ab/ct2, -DNMX_GEMM_BIG=0), two rounds each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
run() { echo "== $*"; timeout -k 10 200 python -u scripts/bench_configs.py "$@" 2>&1 | grep '^{' || exit 1; }
for r in 1 2; do for lib in numpyro_amd/_lib/libnumpyro_amd.so build/ab/ct2/libnumpyro_amd.so; do
  run funnel --chains 4096 --warmup 30 --steps 5 --lib $lib
  run bnn --chains 2048 --warmup 30 --steps 5 --lib $lib
done; done
