"""The reference's structural forms of the initial inverse mass matrix (hmc_util.py:439-487
_initialize_mass_matrix, dict branch; hmc.py:759-769) assembled in ravel coordinates
(numpyro_amd.dense.assemble_inverse_mass_matrix)."""
import numpy as np
import pytest

from numpyro_amd.dense import assemble_inverse_mass_matrix
from numpyro_amd.potentials import POSITIVE, REAL

# eight schools' ravel order: mu (0), tau (1), theta (2..9)
SITES = [("mu", (), REAL), ("tau", (), POSITIVE), ("theta", (8,), REAL)]


def test_dense_group_block_in_group_order():
    rs = np.random.RandomState(0)
    a = rs.randn(9, 9)
    blk = a @ a.T + np.eye(9)  # coordinates (theta_0..7, mu): the group's order
    m = assemble_inverse_mass_matrix(SITES, [("theta", "mu")], {("theta", "mu"): blk, ("tau",): np.array([0.5])})
    m = m.numpy()
    order = list(range(2, 10)) + [0]
    np.testing.assert_array_equal(m[np.ix_(order, order)], blk)
    assert m[1, 1] == 0.5 and np.all(m[1, [0] + list(range(2, 10))] == 0)


def test_missing_blocks_are_identity_and_ones():
    m = assemble_inverse_mass_matrix(SITES, [("theta",)], {}).numpy()
    np.testing.assert_array_equal(m, np.eye(10))


def test_diagonal_forms():
    # dense_mass=False: every dict block diagonal (a matrix contributes its diagonal)
    v = assemble_inverse_mass_matrix(SITES, False, {("theta",): np.diag(np.arange(1.0, 9.0)),
                                                     ("mu",): np.array([3.0])}).numpy()
    np.testing.assert_array_equal(v, np.r_[3.0, 1.0, np.arange(1.0, 9.0)])
    # an array with dense_mass=False: {sorted sites: array} -> its diagonal
    w = assemble_inverse_mass_matrix(SITES, False, np.diag(np.arange(10.0) + 1)).numpy()
    np.testing.assert_array_equal(w, np.arange(10.0) + 1)


def test_dense_true_takes_the_sorted_sites_block():
    rs = np.random.RandomState(1)
    a = rs.randn(10, 10)
    full = a @ a.T + np.eye(10)
    np.testing.assert_array_equal(assemble_inverse_mass_matrix(SITES, True, full).numpy(), full)
    np.testing.assert_array_equal(assemble_inverse_mass_matrix(SITES, True, {("mu", "tau", "theta"): full}).numpy(),
                                  full)


def test_conflicting_groups_raise_like_the_reference():
    with pytest.raises(AssertionError, match="conflict of sites names"):
        # an array with a structured dense_mass becomes {sorted sites: array}: tau, theta, mu twice
        assemble_inverse_mass_matrix(SITES, [("theta", "mu")], np.eye(10))
    with pytest.raises(AssertionError, match="conflict of sites names"):
        assemble_inverse_mass_matrix(SITES, [("theta",)], {("theta", "mu"): np.eye(9)})
