"""Host-side API behaviour (no GPU): the numpyro-shaped constructors validate arguments like
the reference (numpyro/infer/hmc.py:541-948, mcmc.py:224-330), fused models refuse direct
calls, and the engine's host logic (adaptation schedule, fori_collect slot indexing,
dense-mass window segmentation) follows numpyro."""
import math

import numpy as np
import pytest

from numpyro_amd import diagnostics
from numpyro_amd import potentials as P
from numpyro_amd.engine import Engine, build_adaptation_schedule
from numpyro_amd.infer import HMC, MCMC, NUTS
from oracle import hmc_ref as H


def test_kernel_argument_validation():
    with pytest.raises(ValueError):
        NUTS()  # neither model nor potential_fn (hmc.py:570-571)
    with pytest.raises(ValueError):
        NUTS(P.eight_schools, potential_fn=P.DiagNormal([0.0], [1.0]))
    with pytest.raises(ValueError):
        HMC(P.eight_schools, num_steps=None, trajectory_length=None)
    with pytest.raises(TypeError):
        NUTS(3.0)  # a model is a function (front end) or a fused model
    with pytest.raises(NotImplementedError):
        NUTS(lambda: None).potential()  # no sample sites: no fused kernel for this structure
    with pytest.raises(TypeError):
        NUTS(potential_fn=3.0)
    with pytest.raises(ValueError, match="init_params"):  # hmc.py:754-757
        NUTS(potential_fn=lambda z: (z ** 2).sum()).potential()
    with pytest.raises(ValueError):
        NUTS(P.eight_schools, dense_mass=[("mu", 3)])  # groups of site names (hmc.py:239-252)
    with pytest.raises(NotImplementedError):
        NUTS(P.eight_schools, kinetic_fn=lambda m, r: 0.0)
    from numpyro_amd.infer.hmc_util import euclidean_kinetic_energy
    NUTS(P.eight_schools, kinetic_fn=euclidean_kinetic_energy)  # the energy the device integrates
    with pytest.warns(UserWarning):
        HMC(P.eight_schools, num_steps=5, trajectory_length=1.0)  # hmc.py:595-599
    k = NUTS(P.eight_schools, dense_mass=True, max_tree_depth=(8, 10), target_accept_prob=0.9)
    o = k.options()
    assert o.dense_mass and o.max_tree_depth == (8, 10) and o.target_accept_prob == 0.9
    assert k.sample_field == "z" and "diverging" in k.default_fields


def test_mcmc_argument_validation():
    k = NUTS(P.eight_schools)
    with pytest.raises(ValueError):
        MCMC(k, num_warmup=10, num_samples=10, thinning=0)
    with pytest.raises(ValueError):
        MCMC(k, num_warmup=10, num_samples=10, chain_method="pmap")
    m = MCMC(k, num_warmup=10, num_samples=10, num_chains=7, chain_method="vectorized")
    assert (m.chain_lo, m.chain_hi, m.local_chains) == (0, 7, 7)
    m = MCMC(k, num_warmup=10, num_samples=10, num_chains=5, chain_offset=40)
    assert (m.chain_lo, m.chain_hi) == (40, 45)


def test_fused_model_is_not_callable():
    with pytest.raises(TypeError):
        P.eight_schools(8, np.ones(8), np.zeros(8))
    pot = P.eight_schools.potential(8, np.ones(8), np.zeros(8))
    assert pot.dim == 10 and [n for n, _, _ in pot.sites] == ["mu", "tau", "theta"]


def test_potential_site_metadata_follows_ravel_order():
    sv = P.StochasticVolatility(np.ones(20, np.float32))
    assert [n for n, _, _ in sv.sites] == ["nu", "s", "sigma"] and sv.dim == 22
    bnn = P.BNN(np.ones((10, 3), np.float32), np.ones((10, 1), np.float32), 4)
    assert [n for n, _, _ in bnn.sites] == ["prec_obs", "w1", "w2", "w3"]
    assert bnn.dim == 1 + 12 + 16 + 4
    f = P.Funnel(7)
    flat = np.arange(2 * 7, dtype=np.float32).reshape(2, 7)
    out = f.unflatten(flat)
    assert out["x"].shape == (2, 6) and out["y"].shape == (2,)
    np.testing.assert_array_equal(out["y"], flat[:, -1])


@pytest.mark.parametrize("n", [0, 1, 10, 19, 20, 30, 149, 150, 500, 1000, 2345])
def test_adaptation_schedule_matches_oracle(n):
    if n == 0:
        return
    assert build_adaptation_schedule(n) == H.build_adaptation_schedule(n)


def test_fori_collect_slots():
    """numpyro/util.py:330-346: slot (i - start) // thinning, the last write wins."""
    N, lower, thin = 23, 5, 4
    start = lower + (N - lower) % thin
    S = (N - lower) // thin
    slots = {}
    for i in range(N):
        k = Engine._slot_of(i, start, thin, S)
        if k >= 0:
            slots[k] = i
    ref = {}
    for i in range(N):  # the reference loop: every i >= start writes its slot
        if i >= start:
            ref[(i - start) // thin] = i
    assert slots == {k: v for k, v in ref.items() if k < S}


def test_dense_segments_split_at_middle_window_ends():
    class Fake:
        num_warmup = 1000

        class opts:
            adapt_mass_matrix = True

    segs = Engine._dense_segments(Fake(), 0, 2000)
    sched = build_adaptation_schedule(1000)
    middle = [(a, b + 1) for a, b in sched[1:-1]]
    assert [(a, b) for a, b, w in segs if w] == middle
    assert all(w == (a, b) for a, b, w in segs if w)
    assert segs[0] == (0, 75, None) and segs[-1] == (950, 2000, None)
    # contiguous cover
    assert all(segs[i][1] == segs[i + 1][0] for i in range(len(segs) - 1))
    # a run that starts or ends inside a middle window gets the partial piece with its window
    part = Engine._dense_segments(Fake(), 80, 120)
    assert part == [(80, 100, (75, 100)), (100, 120, (100, 150))]
    Fake.opts.adapt_mass_matrix = False
    assert Engine._dense_segments(Fake(), 0, 2000) == [(0, 2000, None)]


def test_host_diagnostics_known_values():
    rs = np.random.RandomState(0)
    iid = rs.randn(4, 4000)
    ess = diagnostics.effective_sample_size(iid)
    assert 0.8 * 16000 < ess < 1.25 * 16000
    assert abs(diagnostics.split_gelman_rubin(iid) - 1.0) < 0.01
    phi = 0.9
    x = np.zeros((4, 20000))
    x[:, 0] = rs.randn(4)
    e = rs.randn(4, 20000)
    for t in range(1, 20000):
        x[:, t] = phi * x[:, t - 1] + e[:, t]
    ess_ar = diagnostics.effective_sample_size(x)
    expected = 80000 * (1 - phi) / (1 + phi)  # AR(1) integrated autocorrelation time
    assert 0.7 * expected < ess_ar < 1.3 * expected
    shifted = np.concatenate([iid[:2], iid[2:] + 3.0])
    assert diagnostics.split_gelman_rubin(shifted) > 1.5
    lo, hi = diagnostics.hpdi(rs.randn(100000), prob=0.9)
    np.testing.assert_allclose([lo, hi], [-1.645, 1.645], atol=0.05)
    assert math.isclose(float(diagnostics.autocorrelation(np.arange(10.0))[0]), 1.0)


def test_pickling_kernels_models_and_states():
    """test/test_pickle.py: samplers, models and states pickle (by reference for model
    functions and fused models, mcmc.py:797-800, hmc.py:818-822); bound device data and the
    engine are left out and rebuilt."""
    import pickle

    import torch

    import model_zoo as Z
    from numpyro_amd.infer.hmc import HMCAdaptState, HMCState

    for model in (P.eight_schools, P.logistic_regression, Z.covtype_model):
        k = pickle.loads(pickle.dumps(NUTS(model, target_accept_prob=0.9)))
        assert k.model is model and k._target_accept_prob == 0.9
    m = MCMC(NUTS(P.funnel), num_warmup=3, num_samples=4, num_chains=6, postprocess_fn=dict)
    m2 = pickle.loads(pickle.dumps(m))
    assert m2.sampler.model is P.funnel and m2.postprocess_fn is dict and m2.num_samples == 4
    # a bound potential pickles without its device data and binds again
    pot = P.DiagNormal([0.0, 1.0], [1.0, 2.0])
    pot.bind(4, 64, "cpu")
    assert hasattr(pot, "prec")
    p2 = pickle.loads(pickle.dumps(pot))
    assert not hasattr(p2, "prec") and not hasattr(p2, "_bound_keys")
    p2.bind(4, 64, "cpu")
    torch.testing.assert_close(p2.prec, pot.prec)
    # a state snapshot: host copies of the arena / whitening, no engine reference
    t = torch.arange(3.0)
    st = HMCState(t, {"x": t}, t, t, t, None, 1.0, t, t, t, t > 1,
                  HMCAdaptState(t, t, t, t, (t,), (t,), t, 7), 7)
    st._arena, st._whitening, st._engine = torch.ones(16, dtype=torch.uint8), (t, None), object()
    st._layout, st._generation = ("DiagNormal", 3, 1, 10, 0, False, False, 1), ("tok", 5)
    st2 = pickle.loads(pickle.dumps(st))
    assert type(st2) is HMCState and st2._engine is None and st2._layout == st._layout
    torch.testing.assert_close(st2._arena, st._arena)
    assert st2.adapt_state.rng_key == 7 and st2._whitening[1] is None


def test_mass_blocks_structure():
    """dense_mass=[("theta", "mu")] on eight schools (sites mu, tau, theta[8]): a dense block over
    theta then mu in the group's order (z_block = tuple(z[k] for k in site_names),
    hmc_util.py:448-456) and a diagonal block over the remaining ("tau",) (:469-477)."""
    import torch

    from numpyro_amd.dense import MassBlocks

    pot = P.eight_schools.potential(8, np.ones(8), np.zeros(8))
    mb = MassBlocks(pot.sites, [("theta", "mu")])
    (g0, i0, d0), (g1, i1, d1) = mb.blocks
    assert g0 == ("theta", "mu") and d0 and i0.tolist() == list(range(2, 10)) + [0]
    assert g1 == ("tau",) and not d1 and i1.tolist() == [1]
    rs = np.random.RandomState(0)
    A = rs.randn(2, 10, 10)
    cov = torch.tensor(A @ A.transpose(0, 2, 1) + 10 * np.eye(10))
    m = mb.mask(cov)
    assert float(m[:, 1, 0].abs().max()) == 0 and float(m[:, 1, 1].min()) > 0 and float(m[:, 0, 2].abs().min()) > 0
    T = mb.factor(m)
    torch.testing.assert_close(T @ T.transpose(-1, -2), m)
    blk = mb.split(m)
    assert blk[("theta", "mu")].shape == (2, 9, 9) and blk[("tau",)].shape == (2, 1)
    # the dense block factor is the reference's flipped Cholesky in the block's own order
    sub = blk[("theta", "mu")].numpy()[0]
    Tb = np.linalg.cholesky(sub[::-1, ::-1])[::-1, ::-1]
    np.testing.assert_allclose(T.numpy()[0][np.ix_(i0.numpy(), i0.numpy())], Tb, rtol=1e-10)
    with pytest.raises(ValueError):
        MassBlocks(pot.sites, [("theta",), ("theta", "mu")])
    with pytest.raises(ValueError):
        MassBlocks(pot.sites, [("beta",)])
    assert NUTS(P.eight_schools, dense_mass=[]).options().dense_mass is False
    o = NUTS(P.eight_schools, dense_mass=[("theta", "mu")]).options()
    assert o.dense_mass is True and o.dense_blocks == [("theta", "mu")]


def test_postprocess_fn_is_applied_per_draw():
    """MCMC(postprocess_fn=fn): fn sees one draw's site values (site-shaped, as the reference's
    fori_collect passes them), so reducing / indexing / reshaping functions give per-draw
    results; a function that cannot be vmapped runs once per draw."""
    import torch

    from numpyro_amd.infer.mcmc import _postprocess_per_draw

    C, S = 3, 4
    g = torch.Generator().manual_seed(0)
    sites = {"theta": torch.randn(C, S, 8, generator=g), "mu": torch.randn(C, S, generator=g)}

    def fn(z):
        return {"s": z["theta"].sum(), "first": z["theta"][0], "m": z["theta"].reshape(2, 4) * z["mu"]}

    out = _postprocess_per_draw(fn, sites)
    assert out["s"].shape == (C, S) and out["first"].shape == (C, S) and out["m"].shape == (C, S, 2, 4)
    torch.testing.assert_close(out["s"], sites["theta"].sum(-1))
    torch.testing.assert_close(out["first"], sites["theta"][..., 0])
    torch.testing.assert_close(out["m"], sites["theta"].reshape(C, S, 2, 4) * sites["mu"][..., None, None])

    def py(z):  # .item(): not vmappable
        return {"s": torch.tensor(float(z["theta"].sum().item()))}

    torch.testing.assert_close(_postprocess_per_draw(py, sites)["s"], sites["theta"].sum(-1))


def test_euclidean_kinetic_energy_matches_oracle():
    """hmc_util.euclidean_kinetic_energy / its gradient (hmc_util.py:1183-1220) against the
    oracle's restatement: diagonal, dense, dict-of-blocks structured mass, dict momenta."""
    import numpy as np
    import torch

    import oracle.hmc_ref as H
    from numpyro_amd.infer.hmc_util import euclidean_kinetic_energy as ke, euclidean_kinetic_grad as kg

    rs = np.random.RandomState(0)
    r = rs.randn(5)
    diag = rs.rand(5) + 0.5
    q = rs.randn(5, 5)
    dense = q @ q.T + np.eye(5)
    for imm in (diag, dense):
        np.testing.assert_allclose(float(ke(torch.tensor(imm), torch.tensor(r))), H.euclidean_kinetic_energy(imm, r),
                                   rtol=1e-12)
        np.testing.assert_allclose(kg(torch.tensor(imm), torch.tensor(r)).numpy(), H.kinetic_grad(imm, r),
                                   rtol=1e-12)
    # structured: {("a", "b"): dense over a (2) and b (1), ("c",): diagonal (2)}; dict momenta
    rd = {"a": torch.tensor(r[:2]), "b": torch.tensor(r[2:3]), "c": torch.tensor(r[3:])}
    blocks = {("a", "b"): torch.tensor(dense[:3, :3]), ("c",): torch.tensor(diag[3:])}
    want = H.euclidean_kinetic_energy(dense[:3, :3], r[:3]) + H.euclidean_kinetic_energy(diag[3:], r[3:])
    np.testing.assert_allclose(float(ke(blocks, rd)), want, rtol=1e-12)


def test_euclidean_kinetic_grad_keeps_the_momentum_structure():
    """_euclidean_kinetic_energy_grad (hmc_util.py:1203-1223) returns M^-1 r in r's pytree shape:
    a dict momentum with a structured (dict-of-blocks) mass gives a {site: grad} dict whose block
    momenta are taken in the group's order (r_block = OrderedDict over site_names), not in sorted
    order; a dict momentum with one dense matrix is unraveled by sorted key (ravel_pytree)."""
    import numpy as np
    import torch

    from numpyro_amd.infer.hmc_util import euclidean_kinetic_grad as kg

    rs = np.random.RandomState(1)
    rd = {"b": torch.tensor(rs.randn(2, 1)), "a": torch.tensor(rs.randn(3)), "c": torch.tensor(rs.randn(2))}
    q = rs.randn(5, 5)
    dense5 = torch.tensor(q @ q.T + np.eye(5))
    # group ("b", "a"): the block's coordinates are b (2) then a (3), against the block as given
    blocks = {("b", "a"): dense5, ("c",): torch.tensor(rs.rand(2) + 0.5)}
    g = kg(blocks, rd)
    assert set(g) == {"a", "b", "c"} and g["b"].shape == (2, 1) and g["a"].shape == (3,)
    v = dense5 @ torch.cat([rd["b"].reshape(-1), rd["a"]])
    torch.testing.assert_close(g["b"].reshape(-1), v[:2])
    torch.testing.assert_close(g["a"], v[2:])
    torch.testing.assert_close(g["c"], blocks[("c",)] * rd["c"])
    # one dense matrix over a dict momentum: sorted-key ravel (a, b, c), unraveled back
    d7 = torch.tensor(np.eye(7) * 2.0 + 0.1)
    g2 = kg(d7, rd)
    flat = torch.cat([rd["a"], rd["b"].reshape(-1), rd["c"]])
    v2 = d7 @ flat
    torch.testing.assert_close(torch.cat([g2["a"], g2["b"].reshape(-1), g2["c"]]), v2)
    assert g2["b"].shape == (2, 1)
    # tuple momentum stays a tuple
    gt = kg(torch.tensor([1.0, 2.0, 3.0]), (torch.tensor([1.0]), torch.tensor([1.0, 1.0])))
    assert isinstance(gt, tuple) and gt[1].tolist() == [2.0, 3.0]


def test_torch_potential_value_and_grad_on_the_host():
    """potential_fn over a pytree (hmc.py:127-130) as a TorchPotential: the site structure comes
    from one chain's init_params (sorted names, ravel_pytree order), U and dU/dz of a batch of
    flat positions from torch.func (vmapped grad_and_value), and a function vmap cannot trace
    (Python control flow on values) falls back to per-chain autograd with the same results."""
    import torch

    from numpyro_amd.infer.hmc import _flatten_init

    def fn(z):
        return 0.5 * (z["b"] ** 2).sum() + (z["a"] - 1.0).pow(2).sum() * 2.0

    ex = {"b": torch.zeros(2, 2), "a": torch.zeros(3)}
    pot = P.TorchPotential(fn, ex)
    assert pot.dim == 7 and [n for n, _, _ in pot.sites] == ["a", "b"] and not pot.array_site
    zc = torch.randn(5, 7)
    u, g = pot._value_and_grad(zc)
    a, b = zc[:, :3], zc[:, 3:]
    torch.testing.assert_close(u, 0.5 * (b ** 2).sum(1) + 2.0 * ((a - 1.0) ** 2).sum(1))
    torch.testing.assert_close(g, torch.cat([4.0 * (a - 1.0), b], 1))
    assert pot._vmap_ok is True

    def branchy(z):  # data-dependent control flow: not vmappable
        return (z ** 2).sum() if float(z[0]) > 0 else (2.0 * z ** 2).sum()

    pb = P.TorchPotential(branchy, torch.zeros(4))
    assert pb.array_site and pb.dim == 4
    zc = torch.tensor([[1.0, 2.0, 0.0, 1.0], [-1.0, 1.0, 1.0, 0.0]])
    u, g = pb._value_and_grad(zc)
    assert pb._vmap_ok is False
    torch.testing.assert_close(u, torch.tensor([6.0, 6.0]))
    torch.testing.assert_close(g, torch.stack([2.0 * zc[0], 4.0 * zc[1]]))
    # init_params: batched dicts / arrays, and one chain's unbatched values
    flat = _flatten_init(pot, {"a": torch.ones(4, 3), "b": torch.zeros(4, 2, 2)}, 4)
    assert flat.shape == (4, 7) and float(flat[:, :3].sum()) == 12.0
    assert _flatten_init(pot, {"a": torch.ones(3), "b": torch.zeros(2, 2)}, 1).shape == (1, 7)
    assert _flatten_init(pb, torch.zeros(4), 1).shape == (1, 4)
    k = NUTS(potential_fn=fn)
    k.bind_potential_fn({"a": torch.ones(6, 3), "b": torch.zeros(6, 2, 2)}, 6)
    assert isinstance(k.potential(), P.TorchPotential) and k.potential().dim == 7
