set -o pipefail
for S in 256 512 1024; do
  echo "S=$S"
  NMX_X3_MAX_SPLITS=$S timeout -k 10 120 python -u scripts/logreg_list_bench.py 36 4096,2048,1024,512,256,128,64,16 || exit 1
done
