# round-4 perf call 1: in-kernel clock of k_logreg_x3 and the 16x16x32 shape probe, tail
# prefetch depth A/B, k_bnn variants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in clock probe16clock; do
  timeout -k 10 120 python -u scripts/x3_clock.py build/ab/$v/libnumpyro_amd.so 4096 || exit 1
done
for r in 1 2; do for v in base probe16; do
  echo "== $v"; timeout -k 10 120 python -u scripts/bench_potential.py d 4096,512 build/ab/$v/libnumpyro_amd.so || exit 1
done; done
timeout -k 10 300 python -u scripts/ab_bnn.py build/ab/bnn_old/libnumpyro_amd.so build/ab/bnn_t32/libnumpyro_amd.so build/ab/bnn_new/libnumpyro_amd.so || exit 1
bash scripts/gpu_r04_ab_tail.sh
