#!/bin/bash
# A/B of the launched wide step (k_wide_v1 / r / s / v2, the dense-mass configs' step) on SV and
# the funnel with diagonal mass forced onto the launched path (scripts/bench_configs.py
# --launched).  usage: scripts/ab_launched_wide.sh variant1 variant2 ...
for v in "$@"; do
  echo "== $v sv8192"
  python -u scripts/bench_configs.py sv --launched --chains 8192 --warmup 50 --steps 10 \
    --lib build/ab/$v/libnumpyro_amd.so 2>&1 | grep '^{' || exit 1
  echo "== $v funnel4096"
  python -u scripts/bench_configs.py funnel --dense 0 --launched --chains 4096 --warmup 30 --steps 5 \
    --lib build/ab/$v/libnumpyro_amd.so 2>&1 | grep '^{' || exit 1
done
