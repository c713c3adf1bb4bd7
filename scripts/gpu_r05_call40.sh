#!/bin/bash
# round 5: the 256 x 128 dense-product tile for launches of >= 256 (instead of >= 512)
# workgroups (BNN c3: 21 x 16 = 336): product A/B and the c3 leg with each build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/call40
mkdir -p $O
timeout -k 10 300 python3 -u scripts/gemm_ab.py numpyro_amd/_lib/libnumpyro_amd.so build/abx/gemm_big256/libnumpyro_amd.so numpyro_amd/_lib/libnumpyro_amd.so build/abx/gemm_big256/libnumpyro_amd.so > $O/gemm_ab.txt 2>&1 || { tail -20 $O/gemm_ab.txt; exit 1; }
grep RESULT $O/gemm_ab.txt
for v in head big256; do
  L=numpyro_amd/_lib/libnumpyro_amd.so; [ $v = big256 ] && L=build/abx/gemm_big256/libnumpyro_amd.so
  timeout -k 10 400 python3 scripts/bench_configs.py bnn --chains 2048 --warmup 100 --steps 5 --lib $L > $O/c3_$v.txt 2>&1 || exit 1
  echo "$v $(grep '^{' $O/c3_$v.txt | tail -1 | cut -c1-260)"
done
