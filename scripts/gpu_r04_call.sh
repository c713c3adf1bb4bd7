set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests/ -m gpu -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/t_all.log 2>&1 ; echo "tests rc $?" >> gpurun_out/t_all.log; tail -3 gpurun_out/t_all.log
