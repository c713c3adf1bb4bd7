#!/bin/bash
# In-run A/B of whole libraries on the headline bench (driver protocol, no CPU leg, no configs),
# alternating the variants.  usage: scripts/ab_headline.sh rounds variant1 variant2 ...
rounds=$1; shift
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    echo "== $v"
    python -u bench.py --steps 20 --warmup 5 --configs none --no-cpu-baseline --lib build/ab/$v/libnumpyro_amd.so \
      2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d[k] for k in ('value', 'potential_ms_per_launch', 'leapfrog_launches', 'mean_tree_size')} | {'frac': d['roofline']['frac']}))" || exit 1
  done
done
