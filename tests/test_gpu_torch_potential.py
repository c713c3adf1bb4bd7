"""A user ``potential_fn`` written with torch operations (numpyro/infer/hmc.py:127-130 -- any
function of a pytree of unconstrained values; the reference differentiates it with
jax.value_and_grad, hmc_util.py:242-252): numpyro_amd.potentials.TorchPotential evaluates it and
its gradient with torch.func on the engine's compacted list (generic path, no fused kernel).

* the same target as a fused kernel (diagonal normal): the same trees and draws to rounding;
* a target no fused kernel covers (a banana), against its known moments;
* init_params required (hmc.py:754-757), array-valued z returned as an array, dense mass."""
import numpy as np
import pytest
import torch

from numpyro_amd import potentials as P
from numpyro_amd.infer import MCMC, NUTS

pytestmark = pytest.mark.gpu

MU = torch.tensor([0.5, -1.0, 2.0, 0.0, 1.5])
SD = torch.tensor([1.0, 0.5, 2.0, 1.5, 0.8])


def diag_fn(z):
    x = z["x"]
    return 0.5 * (((x - MU.to(x.device)) / SD.to(x.device)) ** 2).sum()


def test_torch_potential_matches_the_fused_diag_normal(device):
    """Diagonal normal as a torch potential_fn vs the fused nmx_pe_diag_normal kernel, both
    started from the same init_params on the same Philox stream with a fixed step size (no
    adaptation: rounding differences would otherwise steer the adapted step sizes apart): the
    potentials differ only in float32 rounding, so (nearly) every chain takes the same trees and
    its draws agree to 1e-4."""
    C, W, S = 64, 0, 8
    ip = torch.randn(C, 5, generator=torch.Generator().manual_seed(3))
    runs = []
    kw = dict(step_size=0.4, adapt_step_size=False, adapt_mass_matrix=False)
    for kern in (NUTS(potential_fn=diag_fn, **kw), NUTS(P.diag_normal, **kw)):
        mcmc = MCMC(kern, num_warmup=W, num_samples=S, num_chains=C, progress_bar=False)
        args = () if kern._model is None else (MU.numpy(), SD.numpy())
        init = {"x": ip} if kern._model is None else ip
        mcmc.run(7, *args, init_params=init, extra_fields=("num_steps",))
        runs.append((mcmc.get_samples(True)["x"].cpu().numpy(), mcmc.get_extra_fields(True)["num_steps"].cpu().numpy()))
    (xt, nt), (xf, nf) = runs
    same = np.all(nt[:, :5] == nf[:, :5], axis=1)
    print(f"[torch potential] {same.sum()}/{C} chains take the fused kernel's first 5 trees")
    assert same.sum() >= int(0.9 * C)
    np.testing.assert_allclose(xt[same, :5], xf[same, :5], atol=1e-4, rtol=1e-4)


def test_torch_potential_banana_moments(device):
    """x1 ~ N(0, 1), x2 | x1 ~ N(x1^2 / 2, 1): no fused kernel has this structure.  E[x1] = 0,
    E[x2] = 1/2, Var[x1] = 1, Var[x2] = Var[x1^2] / 4 + 1 = 1.5 (256 chains x 500 draws; the
    tolerances are several standard errors of these estimates at that sample size)."""
    def banana(z):
        x1, x2 = z[0], z[1]
        return 0.5 * x1 ** 2 + 0.5 * (x2 - 0.5 * x1 ** 2) ** 2

    C, S = 256, 500
    mcmc = MCMC(NUTS(potential_fn=banana), num_warmup=500, num_samples=S, num_chains=C, progress_bar=False)
    mcmc.run(11, init_params=torch.zeros(C, 2))
    x = mcmc.get_samples()
    assert torch.is_tensor(x) and x.shape == (C * S, 2)  # an array z comes back as an array
    m = x.double().mean(0).cpu().numpy()
    v = x.double().var(0).cpu().numpy()
    print(f"[banana] mean {m}, var {v}")
    assert abs(m[0]) < 0.05 and abs(m[1] - 0.5) < 0.06
    assert abs(v[0] - 1.0) < 0.1 and abs(v[1] - 1.5) < 0.2


def test_torch_potential_needs_init_params_and_runs_dense(device):
    with pytest.raises(ValueError, match="init_params"):
        MCMC(NUTS(potential_fn=diag_fn), num_warmup=5, num_samples=5, num_chains=4, progress_bar=False).run(0)
    # per-chain dense mass (ChainWhitenedPotential around the torch potential)
    C = 32
    mcmc = MCMC(NUTS(potential_fn=diag_fn, dense_mass=True), num_warmup=150, num_samples=100, num_chains=C,
                progress_bar=False)
    mcmc.run(2, init_params={"x": torch.zeros(C, 5)})
    x = mcmc.get_samples()["x"].double()
    err = (x.mean(0).cpu() - MU.double()).abs() / SD.double()
    print(f"[torch potential dense] standardized mean error {err.numpy()}")
    assert float(err.max()) < 0.15
    imm = mcmc.last_state.adapt_state.inverse_mass_matrix
    assert imm.shape == (C, 5, 5)
