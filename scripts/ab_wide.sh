#!/bin/bash
# A/B of wide-step library builds (scripts/ab_build.py) on the SV config: one rank's share at 8
# GPUs (1024 chains) and the whole config on one GPU (8192 chains).
# usage: scripts/ab_wide.sh variant1 variant2 ...   (build/ab/<variant>/libnumpyro_amd.so)
for ch in 1024 8192; do
  for v in "$@"; do
    echo "== $v $ch"
    python -u scripts/bench_configs.py sv --chains $ch --warmup 50 --steps 10 --lib build/ab/$v/libnumpyro_amd.so 2>&1 \
      | grep '^{' || exit 1
  done
done
