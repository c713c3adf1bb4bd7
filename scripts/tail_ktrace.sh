set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for S in ${SWEEP:-256 512 1024}; do
  NMX_X3_MAX_SPLITS=$S timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tkt$S -o t -- python3 scripts/logreg_list_bench.py 36 16 > gpurun_out/tkt$S.log 2>&1 || exit 1
  rm -f gpurun_out/tkt$S/t_kernel_trace.csv
done
