set -o pipefail
mkdir -p gpurun_out
for sw in ${SWEEP:-default 128 256}; do
  if [ $sw = default ]; then unset NMX_WIDE_SW; else export NMX_WIDE_SW=$sw; fi
  echo "sw=$sw"
  timeout -k 10 200 python -u scripts/bench_configs.py sv --chains 1024 || exit 1
  timeout -k 10 200 python -u scripts/bench_configs.py sv --chains 8192 || exit 1
  timeout -k 10 200 python -u scripts/bench_configs.py funnel --dense 0 || exit 1
done
