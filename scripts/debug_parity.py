"""Debug: print per-transition num_steps / step_size / accept of device vs oracle for a few chains."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from numpyro_amd import datasets
from numpyro_amd import potentials as P
from numpyro_amd.infer import MCMC, NUTS
from oracle import hmc_ref as H, philox, potentials as OP

seed, C, W, S = 1234, 4, 30, 10
args = (8, datasets.EIGHT_SCHOOLS_SIGMA, datasets.EIGHT_SCHOOLS_Y)
mcmc = MCMC(NUTS(P.eight_schools), num_warmup=W, num_samples=S, num_chains=C)
mcmc.warmup(seed, *args, collect_warmup=True, extra_fields=("num_steps", "accept_prob", "adapt_state.step_size", "potential_energy"))
ef = mcmc.get_extra_fields(True)
smp = mcmc.get_samples(True)
ref = OP.EightSchools(datasets.EIGHT_SCHOOLS_Y, datasets.EIGHT_SCHOOLS_SIGMA)
f32 = lambda z: tuple(np.asarray(v, np.float32) for v in ref.pe_grad(z))
for c in range(C):
    o = H.NUTSOracle(f32, 10, W)
    st = o.init(philox.init_uniform(seed, c, 0, 10), seed, c)
    print("chain", c, "init z", st.z[:3], "pe", st.potential_energy)
    for t in range(W):
        st = o.sample(st)
        print(f"  t={t:2d} ns dev={int(ef['num_steps'][c, t])} ora={st.num_steps}  "
              f"acc dev={float(ef['accept_prob'][c, t]):.5f} ora={st.accept_prob:.5f}  "
              f"step dev={float(ef['adapt_state.step_size'][c, t]):.5g} ora={st.adapt_state.step_size:.5g} "
              f"pe dev={float(ef['potential_energy'][c, t]):.5f} ora={st.potential_energy:.5f} "
              f"mu dev={float(smp['mu'][c, t]):.5f} ora={st.z[0]:.5f}")
