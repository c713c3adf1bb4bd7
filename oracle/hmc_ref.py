"""ORACLE (test infrastructure only) — NumPy restatement of numpyro's HMC/NUTS core.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this; the
product (numpyro_amd/) never does.  Every function cites the reference lines it
restates (paths relative to /root/reference).  The reference is JAX-only and cannot run
here: these restatements are pinned by ports of the reference's own
known-answer tests (tests/test_oracle_hmc_util.py <- test/infer/test_hmc_util.py).

Differences from the reference that are deliberate and shared with the engine:
  * randomness comes from `oracle.philox` event streams instead of jax.random.split
    (the reference's stream is unpinned: SURVEY.md §0.5);
  * potentials are (pe, grad) callables with hand-derived gradients instead of
    jax.value_and_grad (hmc_util.py:242-252), see oracle/potentials.py.
Arithmetic is done in `dtype` (float32 by default = the reference's x64-off mode).

Decision margins: when `DECISIONS` is a list, every discrete decision of a trajectory
(transition draws u < p, U-turn angle signs, divergence threshold, HMC accept) appends
(kind, margin) with a scale-free margin, so a parity test can show that a chain whose path
left the oracle's did so at a rounding-level tie (tests/test_gpu_nuts.py).
"""
from __future__ import annotations

import math
import threading
from collections import namedtuple

import numpy as np

from . import philox

DECISIONS = None  # list -> record (kind, margin) of every discrete decision
_TLS = threading.local()  # per-thread log (oracle.cpu_batched runs one chain per thread)


def _log(kind, margin):
    d = getattr(_TLS, "decisions", None)
    if d is None:
        d = DECISIONS
    if d is not None:
        d.append((kind, float(margin)))


def record_decisions(log):
    """Log this thread's decisions into `log` (a list), or stop logging them (None)."""
    _TLS.decisions = log


def record_leaves(log):
    """Append one record per NUTS leaf of this thread's trajectories to `log` (a list of dicts,
    the oracle side of the device's decision trace, nmx_nuts_config.trace), or stop (None).
    A record holds the leaf's delta energy, the in-subtree transition probability and its
    uniform, the smallest iterative U-turn dot checked at the leaf with the magnitude of its
    terms, and, at a subtree end, the biased transition probability, its uniform and the
    whole-tree dot; plus the decisions taken (oracle/parity.py compares them leaf by leaf)."""
    _TLS.leaves = log


def _leaf_log():
    return getattr(_TLS, "leaves", None)


def _angles_scale(inverse_mass_matrix, r_left, r_right, r_sum):
    """(left dot, right dot, scale of each): _momentum_angle's dots and the sums of the
    magnitudes of their terms (the size of their f32 rounding)."""
    v_l = kinetic_grad(inverse_mass_matrix, r_left)
    v_r = kinetic_grad(inverse_mass_matrix, r_right)
    rs = r_sum - (r_left + r_right) / r_sum.dtype.type(2)
    return (float(np.dot(v_l, rs)), float(np.dot(v_r, rs)),
            float(np.dot(np.abs(v_l).astype(np.float64), np.abs(rs))),
            float(np.dot(np.abs(v_r).astype(np.float64), np.abs(rs))))


def _min_dot(pairs):
    """(min dot, its scale) over (dot_l, dot_r, scale_l, scale_r) tuples; (inf, 0) if none."""
    best, sc = math.inf, 0.0
    for dl, dr, sl, sr in pairs:
        if dl < best:
            best, sc = dl, sl
        if dr < best:
            best, sc = dr, sr
    return best, sc


# A decision is a rounding-level tie when device and oracle can order it differently: the
# two compute in f32 with different summation orders (potential, kinetic energy, U-turn
# dots), so energies differ by ~1e-6 relative (dE by ~1e-4 absolute for |E| ~ 1e2-1e3) and
# dot products by ~1e-6 of the magnitude of their terms.  Margins are scale-free (see _log).
TIE = {"transition": 2e-3, "accept": 2e-3, "turn": 1e-3, "diverge": 1e-4}


def tie_score(d):
    kind, m = d
    return m / TIE[kind]


def closest_decision(decisions):
    """The decision of a transition closest to a tie, ("none", inf) without decisions."""
    return min(decisions, key=tie_score) if decisions else ("none", math.inf)


def is_tie(d):
    kind, m = d
    return kind in TIE and m <= TIE[kind]


AdaptWindow = namedtuple("AdaptWindow", ["start", "end"])  # hmc_util.py:16
IntegratorState = namedtuple("IntegratorState", ["z", "r", "potential_energy", "z_grad"])  # :31-33

TreeInfo = namedtuple(  # hmc_util.py:36-57
    "TreeInfo",
    ["z_left", "r_left", "z_left_grad", "z_right", "r_right", "z_right_grad",
     "z_proposal", "z_proposal_pe", "z_proposal_grad", "z_proposal_energy",
     "depth", "weight", "r_sum", "turning", "diverging", "sum_accept_probs", "num_proposals"])

HMCState = namedtuple(  # numpyro/infer/hmc.py:31-48
    "HMCState",
    ["i", "z", "z_grad", "potential_energy", "energy", "r", "trajectory_length",
     "num_steps", "accept_prob", "mean_accept_prob", "diverging", "adapt_state", "rng_key"])

HMCAdaptState = namedtuple(  # hmc_util.py:18-30
    "HMCAdaptState",
    ["step_size", "inverse_mass_matrix", "mass_matrix_sqrt", "mass_matrix_sqrt_inv",
     "ss_state", "mm_state", "window_idx", "rng_key"])


# --------------------------------------------------------------------------- adaptation
def dual_averaging(t0=10, kappa=0.75, gamma=0.05, dtype=np.float32):
    """hmc_util.py:60-130."""
    f = dtype

    def init_fn(prox_center=0.0):
        return (f(0.0), f(0.0), f(0.0), 0, f(prox_center))

    def update_fn(g, state):
        x_t, x_avg, g_avg, t, prox_center = state
        t = t + 1
        g_avg = (f(1) - f(1) / f(t + t0)) * g_avg + f(g) / f(t + t0)  # :117
        x_t = prox_center - f(t ** 0.5) / f(gamma) * g_avg  # :122
        weight_t = f(t ** (-kappa))  # :124
        x_avg = (f(1) - weight_t) * x_avg + weight_t * x_t  # :125
        return (f(x_t), f(x_avg), f(g_avg), t, prox_center)

    return init_fn, update_fn


def welford_covariance(diagonal=True, dtype=np.float32):
    """hmc_util.py:133-239 (array form; dict/structured blocks are not on the hot path)."""

    def init_fn(size):
        shape = (size,) if diagonal else (size, size)
        return (np.zeros(size, dtype), np.zeros(shape, dtype), 0)

    def update_fn(sample, state):
        mean, m2, n = state
        sample = np.asarray(sample, dtype)
        n = n + 1
        delta_pre = sample - mean  # :182
        mean = mean + delta_pre / dtype(n)  # :183
        delta_post = sample - mean
        if m2.ndim == 1:
            m2 = m2 + delta_pre * delta_post  # :186
        else:
            m2 = m2 + np.outer(delta_post, delta_pre)  # :188
        return mean, m2, n

    def final_fn(state, regularize=False):
        mean, m2, n = state
        cov = m2 / dtype(n - 1)  # :212
        if regularize:
            scaled_cov = dtype(n / (n + 5)) * cov  # :215
            shrinkage = dtype(1e-3 * (5 / (n + 5)))  # :216
            if scaled_cov.ndim == 1:
                cov = scaled_cov + shrinkage
            else:
                cov = scaled_cov + shrinkage * np.identity(mean.shape[0], dtype=dtype)
        if cov.ndim == 2:
            # cholesky of the flipped matrix (:224-230)
            flip = cov[::-1, ::-1]
            tril_inv = np.swapaxes(np.linalg.cholesky(flip.astype(np.float64))[::-1, ::-1], -2, -1)
            import scipy.linalg as sla
            cov_inv_sqrt = sla.solve_triangular(tril_inv, np.identity(cov.shape[-1]), lower=True)
            tril_inv = tril_inv.astype(dtype)
            cov_inv_sqrt = cov_inv_sqrt.astype(dtype)
        else:
            tril_inv = np.sqrt(cov).astype(dtype)  # :232
            cov_inv_sqrt = (dtype(1.0) / tril_inv).astype(dtype)  # :233
        return cov.astype(dtype), cov_inv_sqrt, tril_inv

    return init_fn, update_fn, final_fn


def build_adaptation_schedule(num_steps):
    """hmc_util.py:387-436 (Stan windows)."""
    adaptation_schedule = []
    if num_steps < 20:
        adaptation_schedule.append(AdaptWindow(0, num_steps - 1))
        return adaptation_schedule
    start_buffer_size, end_buffer_size, init_window_size = 75, 50, 25
    if (start_buffer_size + end_buffer_size + init_window_size) > num_steps:
        start_buffer_size = int(0.15 * num_steps)
        end_buffer_size = int(0.1 * num_steps)
        init_window_size = num_steps - start_buffer_size - end_buffer_size
    adaptation_schedule.append(AdaptWindow(start=0, end=start_buffer_size - 1))
    end_window_start = num_steps - end_buffer_size
    next_window_size = init_window_size
    next_window_start = start_buffer_size
    while next_window_start < end_window_start:
        cur_window_start, cur_window_size = next_window_start, next_window_size
        if 3 * cur_window_size <= end_window_start - cur_window_start:
            next_window_size = 2 * cur_window_size
        else:
            cur_window_size = end_window_start - cur_window_start
        next_window_start = cur_window_start + cur_window_size
        adaptation_schedule.append(AdaptWindow(cur_window_start, next_window_start - 1))
    adaptation_schedule.append(AdaptWindow(end_window_start, num_steps - 1))
    return adaptation_schedule


def _initialize_mass_matrix(size, inverse_mass_matrix, dense_mass, dtype=np.float32):
    """hmc_util.py:439-515, array branch."""
    if inverse_mass_matrix is None:
        inverse_mass_matrix = np.identity(size, dtype) if dense_mass else np.ones(size, dtype)
        return inverse_mass_matrix, inverse_mass_matrix, inverse_mass_matrix
    inverse_mass_matrix = np.asarray(inverse_mass_matrix, dtype)
    if dense_mass:
        if inverse_mass_matrix.ndim == 1:
            inverse_mass_matrix = np.diag(inverse_mass_matrix)
        flip = inverse_mass_matrix[::-1, ::-1].astype(np.float64)
        mm_sqrt_inv = np.swapaxes(np.linalg.cholesky(flip)[::-1, ::-1], -2, -1)
        import scipy.linalg as sla
        mm_sqrt = sla.solve_triangular(mm_sqrt_inv, np.identity(size), lower=True)
        return inverse_mass_matrix, mm_sqrt.astype(dtype), mm_sqrt_inv.astype(dtype)
    if inverse_mass_matrix.ndim == 2:
        inverse_mass_matrix = np.diag(inverse_mass_matrix).copy()
    mm_sqrt_inv = np.sqrt(inverse_mass_matrix)
    mm_sqrt = dtype(1.0) / mm_sqrt_inv
    return inverse_mass_matrix, mm_sqrt.astype(dtype), mm_sqrt_inv.astype(dtype)


def warmup_adapter(num_adapt_steps, find_reasonable_step_size=None, adapt_step_size=True,
                   adapt_mass_matrix=True, dense_mass=False, target_accept_prob=0.8,
                   regularize_mass_matrix=True, dtype=np.float32):
    """hmc_util.py:518-707."""
    if find_reasonable_step_size is None:
        find_reasonable_step_size = lambda step_size, *args: step_size  # noqa: E731
    ss_init, ss_update = dual_averaging(dtype=dtype)
    mm_init, mm_update, mm_final = welford_covariance(diagonal=not dense_mass, dtype=dtype)
    adaptation_schedule = build_adaptation_schedule(num_adapt_steps)
    num_windows = len(adaptation_schedule)
    f = dtype

    def init_fn(z_info, rng_key, step_size=1.0, inverse_mass_matrix=None, mass_matrix_size=None):
        if mass_matrix_size is None:
            mass_matrix_size = np.size(z_info[0])
        imm, mm_sqrt, mm_sqrt_inv = _initialize_mass_matrix(
            mass_matrix_size, inverse_mass_matrix, dense_mass, dtype)
        if adapt_step_size:
            step_size = find_reasonable_step_size(step_size, imm, z_info, rng_key)
        ss_state = ss_init(np.log(f(10) * f(step_size)))  # :576
        mm_state = mm_init(imm.shape[-1])
        return HMCAdaptState(f(step_size), imm, mm_sqrt, mm_sqrt_inv, ss_state, mm_state, 0, rng_key)

    def _update_at_window_end(z_info, rng_key_ss, state):  # :596-635
        step_size, imm, mm_sqrt, mm_sqrt_inv, ss_state, mm_state, window_idx, rng_key = state
        if adapt_mass_matrix:
            imm, mm_sqrt, mm_sqrt_inv = mm_final(mm_state, regularize=regularize_mass_matrix)
            mm_state = mm_init(imm.shape[-1])
        if adapt_step_size:
            step_size = find_reasonable_step_size(step_size, imm, z_info, rng_key_ss)
            ss_state = ss_init(np.log(f(10)) + np.log(f(step_size)))  # :626
        return HMCAdaptState(step_size, imm, mm_sqrt, mm_sqrt_inv, ss_state, mm_state, window_idx,
                             rng_key)

    def update_fn(t, accept_prob, z_info, state):  # :637-705
        step_size, imm, mm_sqrt, mm_sqrt_inv, ss_state, mm_state, window_idx, rng_key = state
        # a window-end search draws with the next transition's index (device: the chain's
        # iteration counter after transition t)
        rng_key_ss = (rng_key[0], rng_key[1], t + 1) if isinstance(rng_key, tuple) else rng_key
        if adapt_step_size:
            ss_state = ss_update(f(target_accept_prob) - f(accept_prob), ss_state)
            log_step_size, log_step_size_avg = ss_state[0], ss_state[1]
            step_size = np.exp(log_step_size_avg) if t == num_adapt_steps - 1 else np.exp(log_step_size)
            finfo = np.finfo(dtype)
            step_size = f(np.clip(step_size, finfo.tiny, finfo.max))
        is_middle_window = (0 < window_idx) & (window_idx < (num_windows - 1))
        if adapt_mass_matrix:
            z = z_info[0] if isinstance(z_info, (tuple, IntegratorState)) else z_info
            if is_middle_window:
                mm_state = mm_update(np.ravel(z), mm_state)
        t_at_window_end = t == adaptation_schedule[window_idx][1]
        window_idx = window_idx + 1 if t_at_window_end else window_idx
        state = HMCAdaptState(step_size, imm, mm_sqrt, mm_sqrt_inv, ss_state, mm_state, window_idx,
                              rng_key)
        if t_at_window_end and is_middle_window:
            state = _update_at_window_end(z_info, rng_key_ss, state)
        return state

    return init_fn, update_fn


# --------------------------------------------------------------------------- integrator
def euclidean_kinetic_energy(inverse_mass_matrix, r):
    """hmc_util.py:1183-1200."""
    if inverse_mass_matrix.ndim == 2:
        v = inverse_mass_matrix @ r
    else:
        v = inverse_mass_matrix * r
    return r.dtype.type(0.5) * np.dot(v, r)


def kinetic_grad(inverse_mass_matrix, r):
    """hmc_util.py:1203-1220."""
    if inverse_mass_matrix.ndim == 2:
        return inverse_mass_matrix @ r
    return inverse_mass_matrix * r


def velocity_verlet(pe_grad, kinetic_fn=euclidean_kinetic_energy, kinetic_grad_fn=kinetic_grad):
    """hmc_util.py:262-311; pe_grad(z) -> (U, dU/dz) replaces value_and_grad (:242-252)."""

    def init_fn(z, r, potential_energy=None, z_grad=None):
        if potential_energy is None or z_grad is None:
            potential_energy, z_grad = pe_grad(z)
        return IntegratorState(z, r, potential_energy, z_grad)

    def update_fn(step_size, inverse_mass_matrix, state):
        z, r, _, z_grad = state
        half = np.asarray(0.5 * step_size, dtype=np.asarray(r).dtype)
        r = r - half * z_grad  # r(n+1/2), :297-299
        r_grad = kinetic_grad_fn(inverse_mass_matrix, r)
        z = z + np.asarray(step_size, np.asarray(z).dtype) * r_grad  # :301
        potential_energy, z_grad = pe_grad(z)
        r = r - half * z_grad  # :306-308
        return IntegratorState(z, r, potential_energy, z_grad)

    return init_fn, update_fn


def find_reasonable_step_size(pe_grad, kinetic_fn, momentum_generator, init_step_size,
                              inverse_mass_matrix, z_info, rng_key, margins=None):
    """hmc_util.py:314-384; `momentum_generator(z, inverse_mass_matrix, k)` draws the k-th
    attempt's momentum (the reference passes the inverse mass matrix where
    momentum_generator expects its square root, hmc_util.py:359; kept).  `margins` (a list, test
    instrumentation) receives each attempt's (decision margin -dE - log 0.8, energy scale
    |E_current| + |E_new|): a margin within rounding of zero is a tie another float32
    implementation may decide the other way."""
    target_accept_prob = np.float32(np.log(np.float32(0.8)))  # jnp.log(0.8) in float32
    _, vv_update = velocity_verlet(pe_grad, kinetic_fn)
    z, _, potential_energy, z_grad = z_info
    if potential_energy is None or z_grad is None:
        potential_energy, z_grad = pe_grad(z)
    dt = np.asarray(init_step_size).dtype if hasattr(init_step_size, "dtype") else np.float32
    finfo = np.finfo(dt)
    step_size, last_direction, direction = init_step_size, 0, 0
    k = 0

    def cond(step_size, last_direction, direction):
        not_small = (step_size > finfo.tiny) | (direction >= 0)
        not_large = (step_size < finfo.max) | (direction <= 0)
        return (not_small & not_large) & ((last_direction == 0) | (direction == last_direction))

    while cond(step_size, last_direction, direction):
        step_size = (2.0 ** direction) * step_size
        r = momentum_generator(z, inverse_mass_matrix, k)
        k += 1
        _, r_new, potential_energy_new, _ = vv_update(
            step_size, inverse_mass_matrix, (z, r, potential_energy, z_grad))
        energy_current = kinetic_fn(inverse_mass_matrix, r) + potential_energy
        energy_new = kinetic_fn(inverse_mass_matrix, r_new) + potential_energy_new
        delta_energy = energy_new - energy_current
        direction_new = 1 if target_accept_prob < -delta_energy else -1
        if margins is not None:
            margins.append((float(-delta_energy - target_accept_prob), float(abs(energy_current) + abs(energy_new))))
        last_direction, direction = direction, direction_new
    return step_size


# --------------------------------------------------------------------------- NUTS tree
def _momentum_angle(inverse_mass_matrix, r_left, r_right, r_sum):
    """hmc_util.py:710-737."""
    v_left = kinetic_grad(inverse_mass_matrix, r_left)
    v_right = kinetic_grad(inverse_mass_matrix, r_right)
    r_sum = r_sum - (r_left + r_right) / r_sum.dtype.type(2)
    return np.dot(v_left, r_sum), np.dot(v_right, r_sum)


def _is_turning(inverse_mass_matrix, r_left, r_right, r_sum):
    """hmc_util.py:740-746."""
    left_angle, right_angle = _momentum_angle(inverse_mass_matrix, r_left, r_right, r_sum)
    if DECISIONS is not None:  # angle relative to the magnitude of its terms
        v_l = kinetic_grad(inverse_mass_matrix, r_left)
        v_r = kinetic_grad(inverse_mass_matrix, r_right)
        rs = np.abs(r_sum - (r_left + r_right) / r_sum.dtype.type(2))
        _log("turn", min(abs(left_angle) / max(np.dot(np.abs(v_l), rs), 1e-30),
                         abs(right_angle) / max(np.dot(np.abs(v_r), rs), 1e-30)))
    return bool((left_angle <= 0) | (right_angle <= 0))


def _leaf_idx_to_ckpt_idxs(n):
    """hmc_util.py:941-958."""
    idx_max = bin(n >> 1).count("1")
    num_subtrees = bin((~n & (n + 1)) - 1).count("1")
    idx_min = idx_max - num_subtrees + 1
    return idx_min, idx_max


def _is_iterative_turning(inverse_mass_matrix, r, r_sum, r_ckpts, r_sum_ckpts, idx_min, idx_max):
    """hmc_util.py:961-981 (while loop from idx_max down to idx_min, stop at first turn)."""
    r = np.atleast_1d(np.asarray(r))
    r_sum = np.atleast_1d(np.asarray(r_sum))
    r_ckpts = np.asarray(r_ckpts)
    r_sum_ckpts = np.asarray(r_sum_ckpts)
    inverse_mass_matrix = np.asarray(inverse_mass_matrix)
    i, turning = idx_max, False
    while i >= idx_min and not turning:
        subtree_r_sum = r_sum - np.atleast_1d(r_sum_ckpts[i]) + np.atleast_1d(r_ckpts[i])
        turning = _is_turning(inverse_mass_matrix, np.atleast_1d(r_ckpts[i]), r, subtree_r_sum)
        i -= 1
    return turning


class TreeRng:
    """Uniform draws of one NUTS trajectory, keyed like csrc/nmx_common.h events.

    The reference splits keys at hmc_util.py:1161 (direction), :920 (biased transition of
    a doubling) and :1005 (per-leaf uniform transition).
    """

    def __init__(self, seed, chain, it):
        self.seed, self.chain, self.it = seed, chain, it

    def direction(self, j):
        return philox.uniform(self.seed, self.chain, self.it, philox.EV_DIRECTION, j, 0)

    def biased(self, j):
        return philox.uniform(self.seed, self.chain, self.it, philox.EV_BIASED, j, 0)

    def leaf(self, j, k):
        return philox.uniform(self.seed, self.chain, self.it, philox.EV_LEAF, j, k)


def _build_basetree(vv_update, kinetic_fn, z, r, z_grad, inverse_mass_matrix, step_size,
                    going_right, energy_current, max_delta_energy):
    """hmc_util.py:851-894."""
    step_size = step_size if going_right else -step_size
    z_new, r_new, pe_new, z_new_grad = vv_update(step_size, inverse_mass_matrix,
                                                 (z, r, energy_current, z_grad))
    energy_new = pe_new + kinetic_fn(inverse_mass_matrix, r_new)
    delta_energy = energy_new - energy_current
    if np.isnan(delta_energy):
        delta_energy = type(delta_energy)(np.inf)
    tree_weight = -delta_energy
    diverging = bool(delta_energy > max_delta_energy)
    if np.isfinite(delta_energy):
        _log("diverge", abs(delta_energy - max_delta_energy) / max_delta_energy)
    with np.errstate(over="ignore"):
        accept_prob = min(np.exp(-delta_energy), type(delta_energy)(1.0))
    return TreeInfo(z_new, r_new, z_new_grad, z_new, r_new, z_new_grad, z_new, pe_new, z_new_grad,
                    energy_new, 0, tree_weight, r_new, False, diverging, accept_prob, 1)


def _logaddexp(a, b):
    return type(a)(np.logaddexp(a, b))


def _combine_tree(current_tree, new_tree, inverse_mass_matrix, going_right, u, biased_transition):
    """hmc_util.py:767-848; `u` is the transition uniform (random.bernoulli(key, p) = u < p)."""
    if going_right:
        z_left, r_left, z_left_grad = current_tree.z_left, current_tree.r_left, current_tree.z_left_grad
        z_right, r_right, z_right_grad = new_tree.z_right, new_tree.r_right, new_tree.z_right_grad
    else:
        z_left, r_left, z_left_grad = new_tree.z_left, new_tree.r_left, new_tree.z_left_grad
        z_right, r_right, z_right_grad = (current_tree.z_right, current_tree.r_right,
                                          current_tree.z_right_grad)
    r_sum = current_tree.r_sum + new_tree.r_sum
    dt = type(current_tree.weight)
    if biased_transition:  # :756-764, :795-799
        with np.errstate(over="ignore"):
            transition_prob = np.exp(new_tree.weight - current_tree.weight)
        p_raw = transition_prob if np.isnan(transition_prob) else min(transition_prob, dt(1.0))
        transition_prob = dt(0.0) if (new_tree.turning or new_tree.diverging) else min(
            transition_prob, dt(1.0))
        turning = new_tree.turning or _is_turning(inverse_mass_matrix, r_left, r_right, r_sum)
        if _leaf_log() is not None:
            _TLS.last_combine = (float(p_raw), float(u),
                                 _angles_scale(inverse_mass_matrix, r_left, r_right, r_sum))
    else:  # :749-753
        with np.errstate(over="ignore"):
            transition_prob = dt(1.0) / (dt(1.0) + np.exp(-(new_tree.weight - current_tree.weight)))
        turning = current_tree.turning
        if _leaf_log() is not None:
            _TLS.last_combine = (float(transition_prob), float(u), None)
    transition = bool(u < transition_prob)
    if 0.0 < transition_prob < 1.0:
        _log("transition", abs(u - transition_prob))
    src = new_tree if transition else current_tree
    tree_weight = _logaddexp(current_tree.weight, new_tree.weight)
    return TreeInfo(z_left, r_left, z_left_grad, z_right, r_right, z_right_grad,
                    src.z_proposal, src.z_proposal_pe, src.z_proposal_grad, src.z_proposal_energy,
                    current_tree.depth + 1, tree_weight, r_sum, turning, new_tree.diverging,
                    current_tree.sum_accept_probs + new_tree.sum_accept_probs,
                    current_tree.num_proposals + new_tree.num_proposals)


def _get_leaf(tree, going_right):
    """hmc_util.py:897-904."""
    if going_right:
        return tree.z_right, tree.r_right, tree.z_right_grad
    return tree.z_left, tree.r_left, tree.z_left_grad


def _iterative_build_subtree(prototype_tree, vv_update, kinetic_fn, inverse_mass_matrix,
                             step_size, going_right, rng, j, energy_current, max_delta_energy,
                             r_ckpts, r_sum_ckpts):
    """hmc_util.py:984-1085; rng.leaf(j, k) gives the k-th leaf's transition uniform."""
    max_num_proposals = 2 ** prototype_tree.depth
    tree = prototype_tree._replace(num_proposals=0)
    turning = False
    while tree.num_proposals < max_num_proposals and not turning and not tree.diverging:
        z, r, z_grad = _get_leaf(tree, going_right)
        new_leaf = _build_basetree(vv_update, kinetic_fn, z, r, z_grad, inverse_mass_matrix,
                                   step_size, going_right, energy_current, max_delta_energy)
        leaf_idx = tree.num_proposals
        if tree.num_proposals == 0:
            new_tree = new_leaf
            p_leaf, u_leaf, take = -1.0, math.nan, True
        else:
            new_tree = _combine_tree(tree, new_leaf, inverse_mass_matrix, going_right,
                                     rng.leaf(j, leaf_idx), False)
            if _leaf_log() is not None:
                p_leaf, u_leaf, _ = _TLS.last_combine
                take = bool(u_leaf < p_leaf)
        ckpt_idx_min, ckpt_idx_max = _leaf_idx_to_ckpt_idxs(leaf_idx)
        if leaf_idx % 2 == 0:
            r_ckpts[ckpt_idx_max] = new_leaf.r_right
            r_sum_ckpts[ckpt_idx_max] = new_tree.r_sum
        turning = _is_iterative_turning(inverse_mass_matrix, new_leaf.r_right, new_tree.r_sum,
                                        r_ckpts, r_sum_ckpts, ckpt_idx_min, ckpt_idx_max)
        log = _leaf_log()
        if log is not None:
            # every checkpoint dot of the leaf (the loop above stops at the first turning one)
            pairs = [_angles_scale(inverse_mass_matrix, np.atleast_1d(r_ckpts[i]), np.atleast_1d(new_leaf.r_right),
                                   np.atleast_1d(new_tree.r_sum) - np.atleast_1d(r_sum_ckpts[i])
                                   + np.atleast_1d(r_ckpts[i]))
                     for i in range(ckpt_idx_min, ckpt_idx_max + 1)]
            dmin, dscale = _min_dot(pairs)
            n = new_tree.num_proposals
            log.append({"dE": -float(new_leaf.weight), "p_leaf": float(p_leaf), "u_leaf": float(u_leaf),
                        "take_leaf": take, "dot_sub": dmin, "scale_sub": dscale, "turn_sub": bool(turning),
                        "diverge": bool(new_leaf.diverging), "pe": float(new_leaf.z_proposal_pe),
                        "done_sub": bool(n >= max_num_proposals or turning or new_tree.diverging),
                        "p_biased": -1.0, "u_biased": math.nan, "dot_tree": math.inf, "scale_tree": 0.0,
                        "take_biased": False, "turn_tree": False, "iter_done": False, "depth": prototype_tree.depth})
        tree = new_tree
    return tree._replace(depth=prototype_tree.depth, turning=turning)


def build_tree(verlet_update, kinetic_fn, verlet_state, inverse_mass_matrix, step_size, rng,
               max_delta_energy=1000.0, max_tree_depth=10):
    """hmc_util.py:1088-1180."""
    if isinstance(max_tree_depth, tuple):
        max_tree_depth_current, max_tree_depth = max_tree_depth
    else:
        max_tree_depth_current = max_tree_depth
    z, r, potential_energy, z_grad = verlet_state
    energy_current = potential_energy + kinetic_fn(inverse_mass_matrix, r)
    dt = type(energy_current)
    latent_size = np.size(r)
    r_ckpts = np.zeros((max_tree_depth, latent_size), np.asarray(r).dtype)
    r_sum_ckpts = np.zeros((max_tree_depth, latent_size), np.asarray(r).dtype)
    tree = TreeInfo(z, r, z_grad, z, r, z_grad, z, potential_energy, z_grad, energy_current,
                    0, dt(0.0), r, False, False, dt(0.0), 0)
    while tree.depth < max_tree_depth_current and not tree.turning and not tree.diverging:
        j = tree.depth
        going_right = bool(rng.direction(j) < 0.5)
        new_tree = _iterative_build_subtree(tree, verlet_update, kinetic_fn, inverse_mass_matrix,
                                            step_size, going_right, rng, j, energy_current,
                                            max_delta_energy, r_ckpts, r_sum_ckpts)
        tree = _combine_tree(tree, new_tree, inverse_mass_matrix, going_right, rng.biased(j), True)
        log = _leaf_log()
        if log:  # the subtree's last leaf carries the subtree-end decisions
            p_raw, u_b, ang = _TLS.last_combine
            rec = log[-1]
            rec["p_biased"], rec["u_biased"] = p_raw, u_b
            rec["take_biased"] = bool(u_b < (0.0 if (new_tree.turning or new_tree.diverging) else p_raw))
            rec["turn_tree"] = bool(tree.turning)
            if new_tree.num_proposals == 2 ** j and not new_tree.turning and not new_tree.diverging:
                rec["dot_tree"], rec["scale_tree"] = _min_dot([ang])
            rec["iter_done"] = bool(tree.depth >= max_tree_depth_current or tree.turning or tree.diverging)
    return tree


# --------------------------------------------------------------------------- sampler
def momentum_generator(mass_matrix_sqrt, eps):
    """numpyro/infer/hmc.py:92-110 with the noise `eps` supplied."""
    if mass_matrix_sqrt.ndim == 1:
        return mass_matrix_sqrt * eps
    return mass_matrix_sqrt @ eps


class NUTSOracle:
    """One chain of numpyro's NUTS/HMC sample kernel (numpyro/infer/hmc.py:193-530).

    `pe_grad(z) -> (U, dU/dz)`; randomness is keyed by (seed, chain, iteration).
    """

    def __init__(self, pe_grad, dim, num_warmup, *, algo="NUTS", step_size=1.0,
                 adapt_step_size=True, adapt_mass_matrix=True, dense_mass=False,
                 target_accept_prob=0.8, max_tree_depth=10, trajectory_length=2 * math.pi,
                 num_steps=None, regularize_mass_matrix=True, max_delta_energy=1000.0,
                 inverse_mass_matrix=None, find_heuristic_step_size=False, dtype=np.float32):
        self.pe_grad, self.dim, self.num_warmup, self.algo = pe_grad, dim, num_warmup, algo
        self.dtype = dtype
        self.max_delta_energy = max_delta_energy
        self.max_treedepth = (max_tree_depth if isinstance(max_tree_depth, tuple)
                              else (max_tree_depth, max_tree_depth))
        self.trajectory_length = trajectory_length
        self.fixed_num_steps = num_steps
        frs = None
        if find_heuristic_step_size:
            def frs(step_size, inverse_mass_matrix, z_info, rng_key):
                # rng_key = (seed, chain, transition index): attempt k draws Philox event
                # EV_HEURISTIC (csrc/nuts.hip k_heur_propose)
                seed, chain, it = rng_key

                def momentum(z, imm, k):
                    eps = philox.heuristic_normals(seed, chain, it, k, self.dim).astype(dtype)
                    return momentum_generator(np.asarray(imm, dtype), eps).astype(dtype)

                self.search_margins = []
                out = dtype(find_reasonable_step_size(self.pe_grad, euclidean_kinetic_energy, momentum,
                                                      dtype(step_size), inverse_mass_matrix, z_info, None,
                                                      margins=self.search_margins))
                if self.force_search is not None:  # test: teacher-force a search decided at a tie
                    out, self.force_search = dtype(self.force_search), None
                return out
        self.wa_init, self.wa_update = warmup_adapter(
            num_warmup, find_reasonable_step_size=frs, adapt_step_size=adapt_step_size,
            adapt_mass_matrix=adapt_mass_matrix, dense_mass=dense_mass,
            target_accept_prob=target_accept_prob, regularize_mass_matrix=regularize_mass_matrix,
            dtype=dtype)
        self.step_size = step_size
        self.inverse_mass_matrix = inverse_mass_matrix
        self.search_margins, self.force_search = [], None
        self.vv_init, self.vv_update = velocity_verlet(pe_grad)

    def init(self, z, seed, chain):
        """init_kernel (hmc.py:193-362) from a valid unconstrained z."""
        f = self.dtype
        z = np.asarray(z, f)
        pe, z_grad = self.pe_grad(z)
        wa_state = self.wa_init((z, None, pe, z_grad), (seed, chain, 0), f(self.step_size),
                                inverse_mass_matrix=self.inverse_mass_matrix,
                                mass_matrix_size=self.dim)
        return HMCState(0, z, z_grad, pe, None, None, self.trajectory_length, 0, f(0), f(0), False,
                        wa_state, (seed, chain))

    def sample(self, state, it=None):
        """sample_kernel (hmc.py:459-530).  `it` = RNG iteration counter (defaults to state.i)."""
        f = self.dtype
        seed, chain = state.rng_key
        it = state.i if it is None else it
        wa = state.adapt_state
        eps = philox.normals(seed, chain, it, self.dim).astype(f)
        r = momentum_generator(wa.mass_matrix_sqrt, eps).astype(f)
        vv_state = IntegratorState(state.z, r, state.potential_energy, state.z_grad)
        if self.algo == "NUTS":
            depth = self.max_treedepth[0] if state.i < self.num_warmup else self.max_treedepth[1]
            tree = build_tree(self.vv_update, euclidean_kinetic_energy, vv_state,
                              wa.inverse_mass_matrix, wa.step_size, TreeRng(seed, chain, it),
                              max_delta_energy=self.max_delta_energy,
                              max_tree_depth=(depth, max(self.max_treedepth)))
            accept_prob = tree.sum_accept_probs / f(tree.num_proposals)
            num_steps = tree.num_proposals
            vv_state = IntegratorState(tree.z_proposal, vv_state.r, tree.z_proposal_pe,
                                       tree.z_proposal_grad)
            energy, diverging = tree.z_proposal_energy, tree.diverging
        else:
            vv_state, energy, num_steps, accept_prob, diverging = self._hmc_next(
                wa.step_size, wa.inverse_mass_matrix, vv_state, seed, chain, it)
        if state.i < self.num_warmup:
            wa = self.wa_update(state.i, accept_prob, vv_state, wa)
        itr = state.i + 1
        n = itr if state.i < self.num_warmup else itr - self.num_warmup
        mean_accept_prob = state.mean_accept_prob + (accept_prob - state.mean_accept_prob) / f(n)
        return HMCState(itr, vv_state.z, vv_state.z_grad, vv_state.potential_energy, energy, None,
                        state.trajectory_length, num_steps, f(accept_prob), f(mean_accept_prob),
                        bool(diverging), wa, state.rng_key)

    def _hmc_next(self, step_size, inverse_mass_matrix, vv_state, seed, chain, it):
        """hmc.py:364-414."""
        f = self.dtype
        trajectory_length = self.trajectory_length
        if self.fixed_num_steps is not None:
            num_steps = self.fixed_num_steps
        else:
            num_steps = int(np.ceil(f(trajectory_length) / f(step_size)))
        if trajectory_length is not None:
            step_size = f(trajectory_length) / f(num_steps)
        vv_state_new = vv_state
        for _ in range(num_steps):
            vv_state_new = IntegratorState(*self.vv_update(step_size, inverse_mass_matrix,
                                                           vv_state_new))
        energy_old = vv_state.potential_energy + euclidean_kinetic_energy(inverse_mass_matrix,
                                                                          vv_state.r)
        energy_new = vv_state_new.potential_energy + euclidean_kinetic_energy(
            inverse_mass_matrix, vv_state_new.r)
        delta_energy = energy_new - energy_old
        if np.isnan(delta_energy):
            delta_energy = f(np.inf)
        with np.errstate(over="ignore"):
            accept_prob = min(np.exp(-delta_energy), f(1.0))
        diverging = delta_energy > self.max_delta_energy
        u = philox.uniform(seed, chain, it, philox.EV_ACCEPT, 0, 0)
        if accept_prob < 1.0:
            _log("accept", abs(u - accept_prob))
        log = _leaf_log()
        if log is not None:  # one record per HMC transition: the Metropolis decision (device leaf 0)
            log.append({"dE": float(delta_energy), "p_leaf": float(accept_prob), "u_leaf": float(u),
                        "take_leaf": bool(u < accept_prob), "dot_sub": math.inf, "scale_sub": 0.0, "turn_sub": False,
                        "diverge": bool(diverging), "pe": float(vv_state_new.potential_energy), "done_sub": True,
                        "p_biased": -1.0, "u_biased": math.nan, "dot_tree": math.inf, "scale_tree": 0.0,
                        "take_biased": False, "turn_tree": False, "iter_done": True, "depth": 0, "hmc": True})
        if u < accept_prob:
            return vv_state_new, energy_new, num_steps, accept_prob, diverging
        return vv_state, energy_old, num_steps, accept_prob, diverging


def run_chain(pe_grad, z_init, dim, num_warmup, num_samples, seed, chain, **kw):
    """fori_collect over one chain (numpyro/util.py:277-407, progress bar off)."""
    o = NUTSOracle(pe_grad, dim, num_warmup, **kw)
    s = o.init(z_init, seed, chain)
    out = []
    for _ in range(num_warmup + num_samples):
        s = o.sample(s)
        out.append(s)
    return out[num_warmup:], out
