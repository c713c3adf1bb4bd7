"""A/B of library builds on the fused covtype step: the same covtype-shaped NUTS run (logistic
regression D = 55 on 20000 synthetic rows, 256 chains, 50 adaptation + 20 sampling transitions)
in one child process per build; prints each build's draws digest and whether every build's draws
equal the first's bitwise.  usage: python scripts/step_ab.py lib1.so lib2.so ..."""
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys
sys.path.insert(0, @ROOT@)
import numpy as np, torch
from numpyro_amd import native
native.LIB_PATH = @LIB@
from numpyro_amd.infer import MCMC, NUTS
from numpyro_amd import potentials as P
rs = np.random.RandomState(0)
X = rs.randn(20000, 55).astype(np.float32); X[:, -1] = 1.0
y = (rs.rand(20000) < 1 / (1 + np.exp(-X @ (0.3 * rs.randn(55))))).astype(np.float32)
dev = torch.device("cuda:0")
m = MCMC(NUTS(P.logistic_regression), num_warmup=50, num_samples=20, num_chains=256, progress_bar=False)
m.run(3, torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev), extra_fields=("num_steps",))
z = m.get_samples()["coefs"].cpu().numpy()
ns = m.get_extra_fields()["num_steps"].cpu().numpy()
np.save(@OUT@, z)
print("RESULT", int(ns.sum()))
"""


def main():
    digests = []
    for i, lib in enumerate(sys.argv[1:]):
        out = os.path.join(ROOT, "gpurun_out", f"stepab_{i}.npy")
        code = CHILD.replace("@ROOT@", repr(ROOT)).replace("@LIB@", repr(os.path.abspath(lib))).replace(
            "@OUT@", repr(out))
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")]
        if r.returncode or not line:
            print(lib, "FAILED", r.stderr[-2000:])
            sys.exit(1)
        h = hashlib.sha256(open(out, "rb").read()).hexdigest()[:16]
        digests.append(h)
        print(lib, line[0], "draws sha", h, "bitwise equal to the first:", h == digests[0])


if __name__ == "__main__":
    main()
