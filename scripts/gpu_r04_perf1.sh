# round-4 perf call 1: in-kernel clock of k_logreg_x3, tail prefetch depth A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/x3_clock.py build/ab/clock/libnumpyro_amd.so 4096 || exit 1
timeout -k 10 120 python -u scripts/x3_clock.py build/ab/clock/libnumpyro_amd.so 1024 || exit 1
bash scripts/gpu_r04_ab_tail.sh
timeout -k 10 300 python -u scripts/ab_bnn.py build/ab/bnn_old/libnumpyro_amd.so build/ab/bnn_new/libnumpyro_amd.so || exit 1
