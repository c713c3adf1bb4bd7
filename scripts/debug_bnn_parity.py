import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
import test_gpu_nuts as T
rs = np.random.RandomState(321)
args, fm, ref, site, extract, step, frac, z0 = T._fixed_step_case("bnn", 321, rs)
kw = dict(step_size=step, adapt_step_size=False, adapt_mass_matrix=False)
mcmc, warm = T._run_engine(args, fm, 64, 0, 3, 77, init_params=torch.from_numpy(z0), **kw)
ns_dev, sites = T._dev_paths(mcmc, warm)
for c in range(12):
    st = T._oracle_chain(ref.pe_grad, 321, 77, c, 0, 3, z0=z0[c], **kw)
    ns = [s.num_steps for s in st]
    z = extract(np.stack([s.z for s in st]))
    got = sites[site][c].reshape(z.shape)
    print(c, "dev", ns_dev[c].tolist(), "ora", ns, "maxdiff per t", np.abs(got - z).max(axis=1).round(5).tolist(),
          "acc", [round(float(s.accept_prob), 4) for s in st])
