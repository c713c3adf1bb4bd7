"""Ports of the reference's known-answer tests (test/infer/test_hmc_util.py) onto the
NumPy oracle, pinning oracle/hmc_ref.py before it is trusted as the parity checker."""
from collections import namedtuple

import numpy as np
import pytest
from numpy.testing import assert_allclose

from oracle import hmc_ref as H


# test_hmc_util.py:36-52
def test_dual_averaging():
    da_init, da_update = H.dual_averaging(gamma=0.5, dtype=np.float64)
    da_state = da_init()
    for _ in range(10):
        x = da_state[0]
        g = 2 * (x + 1)  # grad of (x + 1)^2
        da_state = da_update(g, da_state)
    assert_allclose(da_state[1], -1.0, atol=1e-3)


# test_hmc_util.py:55-89
@pytest.mark.parametrize("diagonal", [True, False])
@pytest.mark.parametrize("regularize", [True, False])
def test_welford_covariance(diagonal, regularize):
    np.random.seed(0)
    loc = np.random.randn(3)
    a = np.random.randn(3, 3)
    target_cov = a @ a.T
    x = np.random.multivariate_normal(loc, target_cov, size=(2000,))
    wc_init, wc_update, wc_final = H.welford_covariance(diagonal=diagonal, dtype=np.float64)
    st = wc_init(3)
    for i in range(2000):
        st = wc_update(x[i], st)
    cov, cov_inv_sqrt, _ = wc_final(st, regularize=regularize)
    if diagonal:
        diag_cov = np.diagonal(target_cov)
        assert_allclose(cov, diag_cov, rtol=0.06)
        assert_allclose(cov_inv_sqrt, np.sqrt(np.reciprocal(diag_cov)), rtol=0.06)
    else:
        assert_allclose(cov, target_cov, rtol=0.06)
        assert_allclose(cov_inv_sqrt, np.linalg.cholesky(np.linalg.inv(cov)), rtol=0.06)


# test_hmc_util.py:95-229 (velocity_verlet on three analytic systems)
ModelArgs = namedtuple("model_args", ["step_size", "num_steps", "q_i", "p_i", "q_f", "p_f",
                                      "m_inv", "prec"])


def _harmonic(q):
    return 0.5 * q[0] ** 2, np.array([q[0]])


def _planet(q):
    rr = np.sqrt(q[0] ** 2 + q[1] ** 2)
    return -1.0 / rr, q / rr ** 3


def _quartic(q):
    return 0.25 * q[0] ** 4, np.array([q[0] ** 3])


VV_CASES = [
    (_harmonic, ModelArgs(0.01, 100, [0.0], [1.0], [np.sin(1.0)], [np.cos(1.0)], [1.0], 1e-4)),
    (_planet, ModelArgs(0.01, 628, [1.0, 0.0], [0.0, 1.0], [1.0, 0.0], [0.0, 1.0], [1.0, 1.0],
                        5e-3)),
    (_quartic, ModelArgs(0.1, 1810, [0.02], [0.0], [-0.02], [0.0], [1.0], 1e-4)),
]


@pytest.mark.parametrize("pe_grad,args", VV_CASES, ids=["harmonic", "planet", "quartic"])
def test_velocity_verlet(pe_grad, args):
    m_inv = np.array(args.m_inv)
    vv_init, vv_update = H.velocity_verlet(pe_grad)

    def run(q, p):
        st = vv_init(np.array(q, float), np.array(p, float))
        for _ in range(args.num_steps):
            st = vv_update(args.step_size, m_inv, st)
        return st

    st = run(args.q_i, args.p_i)
    assert_allclose(st.z, args.q_f, atol=args.prec)
    assert_allclose(st.r, args.p_f, atol=args.prec)
    e0 = H.euclidean_kinetic_energy(m_inv, np.array(args.p_i, float)) + pe_grad(
        np.array(args.q_i, float))[0]
    e1 = H.euclidean_kinetic_energy(m_inv, st.r) + st.potential_energy
    assert_allclose(e0, e1, atol=1e-5)
    back = run(st.z, -st.r)
    assert_allclose(back.z, args.q_i, atol=1e-4)


# test_hmc_util.py:232-275
@pytest.mark.parametrize("init_step_size", [0.1, 10.0])
def test_find_reasonable_step_size(init_step_size):
    def pe_grad(q):
        return 0.5 * q[0] ** 2, np.array([q[0]])

    p_gen = lambda prototype, m_inv, k: np.array([1.0])  # noqa: E731
    step_size = H.find_reasonable_step_size(pe_grad, H.euclidean_kinetic_energy, p_gen,
                                            np.float64(init_step_size), np.array([1.0]),
                                            (np.array([0.0]), None, None, None), None)
    threshold = np.power(-np.log(0.8) * 8, 0.25)
    if init_step_size < threshold:
        assert step_size / 2 < threshold
        assert step_size > threshold
    else:
        assert step_size * 2 > threshold
        assert step_size < threshold


# test_hmc_util.py:278-292
@pytest.mark.parametrize("num_steps, expected", [
    (18, [(0, 17)]),
    (50, [(0, 6), (7, 44), (45, 49)]),
    (100, [(0, 14), (15, 89), (90, 99)]),
    (150, [(0, 74), (75, 99), (100, 149)]),
    (200, [(0, 74), (75, 99), (100, 149), (150, 199)]),
    (280, [(0, 74), (75, 99), (100, 229), (230, 279)]),
])
def test_build_adaptation_schedule(num_steps, expected):
    assert H.build_adaptation_schedule(num_steps) == [H.AdaptWindow(i, j) for i, j in expected]


# test_hmc_util.py:295-378
def test_warmup_adapter():
    def find_reasonable_step_size(step_size, m_inv, z, rng_key):
        return step_size * 4 if step_size < 1 else step_size / 4

    num_steps = 150
    sched = H.build_adaptation_schedule(num_steps)
    wa_init, wa_update = H.warmup_adapter(num_steps, find_reasonable_step_size, dtype=np.float64)
    z = np.ones(3)
    wa_state = wa_init((z, None, None, None), None, 1.0, mass_matrix_size=3)
    step_size, imm, _, _, _, _, window_idx, _ = wa_state
    assert step_size == find_reasonable_step_size(1.0, imm, z, None)
    assert_allclose(imm, np.ones(3))
    assert window_idx == 0

    w = sched[0]
    for t in range(w.start, w.end + 1):
        wa_state = wa_update(t, 0.7 + 0.1 * t / (w.end - w.start), z, wa_state)
    last = step_size
    step_size, imm, _, _, _, _, window_idx, _ = wa_state
    assert window_idx == 1
    assert step_size < last
    assert_allclose(imm, np.ones(3))

    w = sched[1]
    wl = w.end - w.start
    for t in range(w.start, w.end + 1):
        wa_state = wa_update(t, 0.8 + 0.1 * (t - w.start) / wl, 2 * z, wa_state)
    last = step_size
    step_size, imm, _, _, _, _, window_idx, _ = wa_state
    assert window_idx == 2
    assert step_size > last
    reg = 1e-3 * (5 / (w.end + 1 - w.start + 5))
    assert_allclose(imm, np.full((3,), reg), atol=1e-7)

    w = sched[2]
    for t in range(w.start, w.end + 1):
        wa_state = wa_update(t, 0.8, t * z, wa_state)
    last = step_size
    step_size, final_imm, _, _, _, _, window_idx, _ = wa_state
    assert window_idx == 3
    assert_allclose(step_size, last * 10, atol=1e-6)
    assert_allclose(final_imm, imm)


# test_hmc_util.py:381-386
@pytest.mark.parametrize("leaf_idx, ckpt_idxs",
                         [(0, (1, 0)), (6, (3, 2)), (7, (0, 2)), (13, (2, 2)), (15, (0, 3))])
def test_leaf_idx_to_ckpt_idx(leaf_idx, ckpt_idxs):
    assert H._leaf_idx_to_ckpt_idxs(leaf_idx) == ckpt_idxs


# test_hmc_util.py:389-403
@pytest.mark.parametrize("ckpt_idxs, expected_turning",
                         [((3, 2), False), ((3, 3), True), ((0, 0), False), ((0, 1), True),
                          ((1, 3), True)])
def test_is_iterative_turning(ckpt_idxs, expected_turning):
    actual = H._is_iterative_turning(np.ones(1), 1.0, 3.0, np.array([1.0, 2.0, 3.0, -2.0]),
                                     np.array([2.0, 4.0, 4.0, -1.0]), *ckpt_idxs)
    assert expected_turning == actual


# test_hmc_util.py:406-442
@pytest.mark.parametrize("step_size", [0.01, 1.0, 100.0])
@pytest.mark.parametrize("chain", [0, 1, 2])
def test_build_tree(step_size, chain):
    def pe_grad(q):
        return np.float32(0.5) * q[0] ** 2, q.copy()

    vv_init, vv_update = H.velocity_verlet(pe_grad)
    vv_state = vv_init(np.zeros(1, np.float32), np.ones(1, np.float32))
    tree = H.build_tree(vv_update, H.euclidean_kinetic_energy, vv_state, np.ones(1, np.float32),
                        np.float32(step_size), H.TreeRng(0, chain, 0))
    assert tree.num_proposals >= 2 ** (tree.depth - 1)
    assert tree.sum_accept_probs <= tree.num_proposals
    if tree.depth < 10:
        assert tree.turning | tree.diverging
    if step_size > 10:
        assert tree.diverging
        assert tree.num_proposals == 1
    if step_size < 0.1:
        assert tree.num_proposals > 10
