"""k_gemm_x3 alone (the dense-mass whitening product of BASELINE config 2): the upper
triangular D x D split-bf16 product on C chains, timed with events; for rocprof PMC passes.
    python scripts/bench_gemm_x3.py [D] [C] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.bench_configs import bench_gemm  # noqa: E402

if __name__ == "__main__":
    D = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    bench_gemm(D, C, reps=reps, tri=1, x3=True)
