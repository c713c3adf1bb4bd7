"""Host driver of the device NUTS/HMC state machine (csrc/nuts.hip).

All chain state lives in one device arena (a torch uint8 tensor) laid out by the library;
this module owns the arena, the collection buffers and the launch loop

    nuts_step -> [potential -> nuts_step] * n      (until every chain is DONE)

and never touches chain state on the host.  It corresponds to the reference's
``fori_collect`` loop over ``sample_kernel`` (numpyro/util.py:277-407,
numpyro/infer/hmc.py:459-530) with ``progress_bar=False``.
"""
from __future__ import annotations

import contextlib
import ctypes
import math
import uuid
from dataclasses import dataclass

import torch

from . import native
from .native import NutsConfig, EvalBatch, check, lib, ptr, stream_ptr

INIT_ATTEMPTS = 100  # find_valid_initial_params (numpyro/infer/util.py:386-388)

# ids of arena contents (Engine.generation): (process token, counter), so a state pickled in
# another process never matches a generation of this one
_PROCESS_TOKEN = uuid.uuid4().hex
_counter = iter(range(1, 1 << 62))
_generations = ((_PROCESS_TOKEN, n) for n in _counter)


def build_adaptation_schedule(num_steps):
    """Stan windows, numpyro/infer/hmc_util.py:387-436 (host-side; sent to the device)."""
    schedule = []
    if num_steps < 20:
        schedule.append((0, num_steps - 1))
        return schedule
    start_buffer, end_buffer, init_window = 75, 50, 25
    if start_buffer + end_buffer + init_window > num_steps:
        start_buffer = int(0.15 * num_steps)
        end_buffer = int(0.1 * num_steps)
        init_window = num_steps - start_buffer - end_buffer
    schedule.append((0, start_buffer - 1))
    end_window_start = num_steps - end_buffer
    next_size, next_start = init_window, start_buffer
    while next_start < end_window_start:
        cur_start, cur_size = next_start, next_size
        if 3 * cur_size <= end_window_start - cur_start:
            next_size = 2 * cur_size
        else:
            cur_size = end_window_start - cur_start
        next_start = cur_start + cur_size
        schedule.append((cur_start, next_start - 1))
    schedule.append((end_window_start, num_steps - 1))
    return schedule


@dataclass
class SamplerOptions:
    algo: int = native.ALGO_NUTS
    step_size: float = 1.0
    adapt_step_size: bool = True
    adapt_mass_matrix: bool = True
    dense_mass: bool = False
    target_accept_prob: float = 0.8
    max_tree_depth: tuple = (10, 10)
    trajectory_length: float | None = 2 * math.pi
    num_steps: int | None = None
    regularize_mass_matrix: bool = True
    max_delta_energy: float = 1000.0
    inverse_mass_matrix: object = None  # diag [D], dense [D, D], {site group: block} or None
    # dense pooled adaptation: bytes of window draws buffered per chunk
    dense_adapt_bytes: int = 4 << 30
    # per-chain dense mass: device bytes allowed for the matrices (dense.chain_dense_bytes)
    chain_dense_bytes: int = 64 << 30
    find_heuristic_step_size: bool = False
    # structured mass (dense_mass=[("x", "y"), ...], hmc.py:239-252): site groups of the dense
    # blocks; the remaining sites form one diagonal block
    dense_blocks: list | None = None


class Engine:
    """Chains of one device: arena + potential + launch loop."""

    # one-launch persistent schedule for one-wave models (False: the launched loop; tests
    # compare the two)
    persistent = True
    # D-split models: the step fused with the potential (nmx_nuts_step_wide_model; False: the
    # launched potential + step loop, which tests compare it with)
    fused_wide = True
    # D-split models with diagonal mass: the persistent per-chain schedule (nmx_nuts_run_wide,
    # chain-row arena layout); False: the launched wide schedules above
    wide_persistent = True
    # D-split models behind a batched (dense-mass) potential: the launched loop with the
    # per-chain step kernel on a chain-row arena (k_chain_step); False: the D-slice kernels
    chain_rows_step = True
    # launched fused step (dim <= 256): chain groups stepped on their own streams so that one
    # group's latency-bound step and potential tail overlap another group's potential
    # (nmx_nuts_config.num_groups; 1: one stream).  Measured slower for covtype (each group's
    # potential streams the whole X: 512 chains 0.745M / 0.673M leapfrog/s at 2 / 4 groups vs
    # 0.875M, 4096 chains 1.322M / 1.263M vs 1.369M; profiles/r03/ab_chain_groups.txt): off.
    chain_groups = 1

    def __init__(self, potential, num_chains: int, opts: SamplerOptions, device=None,
                 chain_offset: int = 0, sync_chains: bool = False):
        self.dense = bool(opts.dense_mass)
        self.model_potential = potential
        # the initial inverse mass matrix in ravel coordinates: a dict of site-group blocks, a
        # structured dense_mass's array, or a matrix for a diagonal mass take the reference's
        # structural form (hmc_util.py:439-487)
        imm = opts.inverse_mass_matrix
        # a plain array is in the reference's ravel_pytree order (sorted site names); the
        # potential's layout may order its sites otherwise (front-end models renamed by their
        # own site names): remap it then, so a vector and a matrix land on the same coordinates
        layout_sorted = [n for n, _, _ in potential.sites] == sorted(n for n, _, _ in potential.sites)
        if imm is not None and (isinstance(imm, dict) or opts.dense_blocks or not layout_sorted or
                                (not self.dense and torch.as_tensor(imm).dim() == 2)):
            from .dense import assemble_inverse_mass_matrix
            structure = opts.dense_blocks if opts.dense_blocks else self.dense
            imm = assemble_inverse_mass_matrix(potential.sites, structure, imm)
        self.init_inverse_mass_matrix = imm
        # dense mass: per-chain matrices (the reference's semantics) when they are adapted and
        # fit, one pooled matrix when asked for ("pooled"), one shared whitening when the
        # matrix is given and not adapted (every chain holds the same one: same semantics);
        # structured blocks are always per chain (each block factored in its own order)
        self.chain_dense = self.dense and opts.dense_mass != "pooled" and (bool(opts.adapt_mass_matrix)
                                                                           or bool(opts.dense_blocks))
        self.blocks = None
        if opts.dense_blocks:
            # structured mass: per chain (the reference's semantics), or pooled over chains
            # (dense_mass=pooled([...]): one block-structured matrix, WhitenedPotential below)
            from .dense import MassBlocks
            self.blocks = MassBlocks(potential.sites, opts.dense_blocks)
        if self.chain_dense:
            from .dense import CHAIN_DENSE_MAX_D, ChainWhitenedPotential, chain_dense_bytes
            need = chain_dense_bytes(potential.dim, num_chains)
            if potential.dim > CHAIN_DENSE_MAX_D or need > opts.chain_dense_bytes:
                raise ValueError(
                    f"per-chain dense mass matrices for {num_chains} chains of dimension {potential.dim} need "
                    f"{need / 2**30:.1f} GiB (limit {opts.chain_dense_bytes / 2**30:.0f} GiB, dim <= "
                    f"{CHAIN_DENSE_MAX_D}); use " + ("numpyro_amd.infer.pooled(dense_mass)" if self.blocks is not None
                                                     else "dense_mass='pooled'") +
                    " for one matrix adapted over all chains")
            potential = ChainWhitenedPotential(potential, self.blocks)
        elif self.dense:
            from .dense import WhitenedPotential
            potential = WhitenedPotential(potential, self.blocks)
        self.potential = potential
        self.C = int(num_chains)
        self.D = int(potential.dim)
        self.opts = opts
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.ldc = (self.C + 63) // 64 * 64
        self.md = max(opts.max_tree_depth) if opts.algo == native.ALGO_NUTS else 1
        if self.md > native.MAX_TREE_DEPTH:
            raise ValueError(f"max_tree_depth {self.md} > {native.MAX_TREE_DEPTH}")
        self.chain_offset = int(chain_offset)
        self.sync_chains = bool(sync_chains)
        self.iter_capacity = 1
        self.arena = None
        self._views = {}
        self.iteration = 0  # transitions completed by every chain
        self.num_warmup = 0
        # id of the arena's current contents: a state snapshot taken at this generation can
        # be resumed without copying the arena back (MCMC.run after warmup, kernel.sample)
        self.generation = None
        self._pool = None  # dense pooled adaptation: (window, PooledCovariance) across run() calls
        self._wide_ws = None  # nmx_nuts_step_wide_model workspace (zero-filled once)
        self._side_streams = []  # chain groups 1.. (created on first use)
        self._mass_cache = None  # dense: (whitening version, HMCAdaptState mass fields)
        # False: collected draws stay unconstrained (MCMC(postprocess_fn=...) maps them itself)
        self.constrain_samples = True
        self._trace = None  # per-leaf decision trace (set_trace), off by default
        # (shard.DeviceGroup, rank) when this engine is one device of a process's multi-device
        # run (MCMC chain_method="parallel"): pooled dense moments are summed over the group
        self.device_group = None
        self.cfg = NutsConfig()
        self.potential.bind(self.C, self.ldc, self.device)
        # chain-row arena layout for the persistent wide schedule (decided once: the arena's
        # layout is part of a resumable state).  The step-size search runs on the launched
        # kernels, which index [D][ldc]: with it, the launched schedule.
        wide = lib().nmx_nuts_num_slices(self.D) > 0 and not opts.find_heuristic_step_size
        self.persist_wide = (self.wide_persistent and wide and not self.dense
                             and getattr(self.potential, "wide_model", None) is not None
                             and self.potential.wide_model() is not None)
        self.crow = self.persist_wide or (self.chain_rows_step and wide and self.dense and not self.chain_dense)
        if self.dense and not self.chain_dense:
            self.potential.rows = self.crow  # the whitening packs the listed chains' rows

    # ------------------------------------------------------------------ arena
    def _alloc(self, iter_capacity: int):
        self.iter_capacity = max(1, int(iter_capacity))
        nbytes = lib().nmx_nuts_arena_bytes(self.C, self.D, self.md, self.iter_capacity)
        self.arena = torch.zeros(nbytes, dtype=torch.uint8, device=self.device)
        self._views = {}
        z, g, pe, ph = (ptr(self.view(n)) for n in ("z_eval", "g_eval", "pe_eval", "phase"))
        idx = self.view("active_idx")
        cnt = self.view("counters")
        # dense batch (init: every chain with phase >= LEAF) and the two compacted lists
        self.eval_batch = EvalBatch(z=z, grad=g, pe=pe, phase=ph, active_idx=None, active_count=None,
                                    num_chains=self.C, ldc=self.ldc)
        self.eval_lists = [EvalBatch(z=z, grad=g, pe=pe, phase=ph, active_idx=ptr(idx) + 4 * p * self.ldc,
                                     active_count=ptr(cnt) + 4 * (2 + p), num_chains=self.C, ldc=self.ldc)
                           for p in (0, 1)]

    def view(self, name: str):
        """torch view of an arena field: scalars [ldc], vectors [D, ldc], ckpts [md, D, ldc]."""
        if name in self._views:
            return self._views[name]
        off, nb = ctypes.c_size_t(), ctypes.c_size_t()
        check(lib().nmx_nuts_field_info(self.C, self.D, self.md, self.iter_capacity,
                                        native.FIELD_ID[name], ctypes.byref(off), ctypes.byref(nb)))
        raw = self.arena[off.value:off.value + nb.value]
        t = raw.view(torch.int32 if name in native.INT_FIELDS else torch.float32)
        if name in native.VECTOR_FIELDS:
            # chain-row layout: stored [ldc][D], viewed [D, ldc] like the other layout
            t = t.view(self.ldc, self.D).t() if self.crow else t.view(self.D, self.ldc)
        elif name in native.CKPT_FIELDS:
            t = t.view(self.md, self.ldc, self.D).transpose(1, 2) if self.crow else t.view(self.md, self.D, self.ldc)
        self._views[name] = t
        return t

    # ------------------------------------------------------------------ config
    def _fill_cfg(self, iter_begin, iter_end, num_warmup, seed, collect_start, thinning, collection_size):
        o, c = self.opts, self.cfg
        c.algo = o.algo
        c.num_chains = self.C
        c.dim = self.D
        c.max_depth_alloc = self.md
        d1, d2 = o.max_tree_depth
        c.max_tree_depth_warmup = int(d1)
        c.max_tree_depth = int(d2)
        c.num_warmup = int(num_warmup)
        c.iter_begin = int(iter_begin)
        c.iter_end = int(iter_end)
        c.iter_capacity = self.iter_capacity
        c.adapt_step_size = int(bool(o.adapt_step_size))
        # dense mass: identity on the device (whitened coordinates), pooled on the host side
        c.adapt_mass_matrix = int(bool(o.adapt_mass_matrix) and not self.dense)
        c.regularize_mass_matrix = int(bool(o.regularize_mass_matrix))
        c.unit_mass = int(self.dense or (not o.adapt_mass_matrix and o.inverse_mass_matrix is None))
        c.sync_chains = int(self.sync_chains)
        c.target_accept_prob = float(o.target_accept_prob)
        c.max_delta_energy = float(o.max_delta_energy)
        c.trajectory_length = float(o.trajectory_length) if o.trajectory_length is not None else -1.0
        c.num_steps = int(o.num_steps) if o.num_steps is not None else 0
        sched = build_adaptation_schedule(int(num_warmup)) if num_warmup > 0 else [(0, -1)]
        if len(sched) > native.MAX_WINDOWS:
            raise ValueError("too many adaptation windows")
        c.num_windows = len(sched)
        for i in range(native.MAX_WINDOWS):
            c.window_end[i] = sched[i][1] if i < len(sched) else -1
        c.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        c.chain_offset = self.chain_offset
        c.collect_start = int(collect_start)
        c.collect_thinning = int(thinning)
        c.collection_size = int(collection_size)
        c.ldc = self.ldc
        c.layout = native.LAYOUT_CHAIN_ROWS if self.crow else native.LAYOUT_CHAIN_MINOR
        tr = self._trace
        if tr is None:
            c.trace, c.trace_chains, c.trace_it0, c.trace_iters, c.trace_leaves = None, 0, 0, 0, 0
        else:
            c.trace = ptr(tr["buf"])
            c.trace_chains, c.trace_it0 = tr["chains"], tr["it0"]
            c.trace_iters, c.trace_leaves = tr["buf"].shape[0], tr["buf"].shape[2]

    # ------------------------------------------------------------------ decision trace
    def set_trace(self, chains: int, it0: int, iters: int):
        """Record the per-leaf decision quantities (nmx_nuts_config.trace, enum nmx_trace_field)
        of arena chains [0, chains) for transitions [it0, it0 + iters) of later runs; results do
        not change.  Used by the parity tests and bench.py's parity legs to locate the leaf at
        which a device transition first parts from the oracle's (oracle/parity.py)."""
        if chains <= 0 or iters <= 0:
            self._trace = None
            return
        leaves = 1 << self.md
        buf = torch.full((int(iters), min(int(chains), self.C), leaves, native.TRACE_REC), float("nan"),
                         dtype=torch.float32, device=self.device)
        self._trace = {"buf": buf, "chains": buf.shape[1], "it0": int(it0)}

    def trace_records(self):
        """The decision trace as a float32 numpy array [iters, chains, leaves, TRACE_REC] (NaN:
        no leaf recorded), or None."""
        if self._trace is None:
            return None
        return self._trace["buf"].cpu().numpy()

    # ------------------------------------------------------------------ phases
    def initialize(self, seed: int, num_warmup: int, init_params=None, radius: float = 2.0,
                   stream=None):
        """Reset adaptation state and find a valid initial point for every chain
        (HMC.init -> initialize_model / find_valid_initial_params + init_kernel)."""
        s = stream_ptr(stream)
        # the arena is about to change: no earlier snapshot may take the no-copy resume
        # shortcut, even if the initial-point search below raises
        self.generation = next(_generations)
        self.num_warmup = int(num_warmup)
        self._alloc(self.iter_capacity)
        self._fill_cfg(0, 0, num_warmup, seed, 0, 1, 0)
        imm = self.init_inverse_mass_matrix
        imm_t = None
        if self.dense:
            # chains are initialised in model coordinates (w = z), then re-expressed
            self.potential.whitening.set(torch.eye(self.D, dtype=torch.float64),
                                         None if self.chain_dense else torch.zeros(self.D))
        elif imm is not None:
            imm_t = torch.as_tensor(imm, dtype=torch.float32, device=self.device).reshape(-1)
            if imm_t.numel() != self.D:
                raise ValueError("inverse_mass_matrix must be a diagonal of size D")
        check(lib().nmx_nuts_reset(ctypes.byref(self.cfg), ptr(self.arena), float(self.opts.step_size),
                                   ptr(imm_t), s), "nmx_nuts_reset")
        if init_params is not None:
            z = torch.as_tensor(init_params, dtype=torch.float32, device=self.device)
            z = z.reshape(self.C, self.D)
            zt = torch.zeros(self.D, self.ldc, dtype=torch.float32, device=self.device)
            zt[:, :self.C] = z.t()
            check(lib().nmx_nuts_init_from(ctypes.byref(self.cfg), ptr(self.arena), ptr(zt), s))
            self._evaluate_all(s)
            check(lib().nmx_nuts_init_check(ctypes.byref(self.cfg), ptr(self.arena), s))
            bad = int(self.view("counters")[1].item())
            if bad:
                raise RuntimeError(f"Cannot find valid initial parameters: {bad} chains have "
                                   "non-finite potential energy or gradient at init_params.")
        else:
            for attempt in range(INIT_ATTEMPTS):
                check(lib().nmx_nuts_init_draw(ctypes.byref(self.cfg), ptr(self.arena), attempt,
                                               float(radius), s))
                self._evaluate_all(s)
                check(lib().nmx_nuts_init_check(ctypes.byref(self.cfg), ptr(self.arena), s))
                if int(self.view("counters")[1].item()) == 0:
                    break
            else:
                raise RuntimeError("Cannot find valid initial parameters. Please check your model "
                                   "again.")  # infer/util.py:795-797
        self.iteration = 0
        self._pool = None
        if self.dense and imm is not None:
            self._reexpress(imm, None, s)
        if self._heuristic():
            self._find_step_size(True, s)
        self.generation = next(_generations)

    def _evaluate_all(self, s):
        """The potential at z_eval of every chain with phase >= LEAF (initial points).  The
        potential kernels take [D][ldc] positions: a chain-row arena is evaluated through
        transposed copies."""
        if not self.crow:
            self.potential.evaluate(self.eval_batch, s)
            return
        zt = self.view("z_eval").contiguous()
        gt = torch.zeros_like(zt)
        b = EvalBatch(z=ptr(zt), grad=ptr(gt), pe=ptr(self.view("pe_eval")), phase=ptr(self.view("phase")),
                      active_idx=None, active_count=None, num_chains=self.C, ldc=self.ldc)
        self.potential.evaluate(b, s)
        self.view("g_eval").copy_(gt)

    # ------------------------------------------------------------------ dense mass
    def _heuristic(self):
        # wa_init searches whenever adapt_step_size is set, num_warmup = 0 included
        # (hmc.py:319-339 -> hmc_util.py:572-576); the window-end searches exist only with
        # middle windows (_window_ends is empty without warmup)
        o = self.opts
        return bool(o.find_heuristic_step_size) and bool(o.adapt_step_size)

    def _find_step_size(self, at_init, s):
        """find_reasonable_step_size for every chain from its stored state (warmup_adapter at
        init, hmc_util.py:573-576, and at middle-window ends, :619-626): rounds of propose ->
        potential on the searching chains -> finish until no chain searches."""
        L = lib()
        cfgp = ctypes.byref(self.cfg)
        arena = ptr(self.arena)
        ev = self.eval_lists[0]
        ev.num_chains = self.C
        check(L.nmx_heuristic_begin(cfgp, arena, s), "nmx_heuristic_begin")
        eps = torch.zeros(self.D, self.ldc, dtype=torch.float32, device=self.device) if self.dense else None
        for _ in range(600):  # the step doubles or halves each round: <= 2 x 254 rounds to an extreme
            if self.dense:
                check(L.nmx_heuristic_noise(cfgp, arena, ptr(eps), s), "nmx_heuristic_noise")
                check(L.nmx_heuristic_propose_with(cfgp, arena, ptr(self._dense_momentum(eps, s)), s),
                      "nmx_heuristic_propose_with")
            else:
                check(L.nmx_heuristic_propose(cfgp, arena, s), "nmx_heuristic_propose")
            self.potential.evaluate(ev, s)
            check(L.nmx_heuristic_finish(cfgp, arena, int(at_init), s), "nmx_heuristic_finish")
            if int(self.view("counters")[1].item()) == 0:
                return
        raise RuntimeError("find_reasonable_step_size did not terminate")

    def _dense_momentum(self, eps, s):
        """The search's momentum in whitened coordinates, p = T^T M^-1 eps = T^T T T^T eps:
        the reference draws r = M^-1 eps (hmc_util.py:359, momentum_generator called with the
        inverse mass matrix) and moves z by M^-1 r; with z = mu + T w that is w' = p = T^T r
        and kinetic 0.5 r^T M^-1 r = 0.5 |p|^2.  Three device products (the pooled GEMMs or
        the per-chain matvecs) on [D, ldc]."""
        wt = self.potential.whitening
        a, b = torch.empty_like(eps), torch.empty_like(eps)
        if self.chain_dense:
            for fwd, x, o in ((False, eps, a), (True, a, b), (False, b, a)):
                wt.matvec(fwd, ptr(x), ptr(o), None, None, None, self.C, self.ldc, s)
        else:
            for fwd, x, o in ((False, eps, a), (True, a, b), (False, b, a)):
                wt.product(fwd, ptr(x), ptr(o), None, None, None, self.C, self.ldc, s)
        return a

    def _search_at_window_end(self, e, cstart, thinning, S, fields, s):
        """find_reasonable_step_size at the end of a middle window (hmc_util.py:619-626); the
        transition that ended the window reports the searched step size, as its adapt_state
        does in the reference (update_fn returns it, :700-705)."""
        self._find_step_size(False, s)
        slot = self._slot_of(e - 1, cstart, thinning, S)
        if slot >= 0:
            fields[slot, native.COLLECT.index("step_size"), :self.C] = self.view("step_size")[:self.C]

    def _search_cuts(self, a, b):
        """Window ends e in (a, b] at which the step-size search runs (sorted)."""
        return [e for e in self._window_ends() if a < e <= b] if self._heuristic() else []

    def _window_ends(self):
        """First transition index after each middle adaptation window (hmc_util.py:596-635)."""
        sched = build_adaptation_schedule(self.num_warmup)
        return [we + 1 for i, (_, we) in enumerate(sched) if 0 < i < len(sched) - 1]

    def _reexpress(self, inverse_mass_matrix, mu, s):
        """Change the whitening of every chain (at an iteration boundary): z is kept,
        w = T_new^-1 (z - mu_new), and U, grad_w are re-evaluated at the new w."""
        wt = self.potential.whitening
        z = torch.empty(self.D, self.ldc, dtype=torch.float32, device=self.device)
        wt.to_model(self.view("z").contiguous(), z, stream=s)
        w = torch.zeros(self.D, self.ldc, dtype=torch.float32, device=self.device)
        lock = self.device_group[0].linalg_lock if self.device_group is not None else contextlib.nullcontext()
        with lock:
            wt.set(inverse_mass_matrix, mu)
            w[:, :self.C] = wt.to_whitened(z[:, :self.C])
            torch.cuda.current_stream(self.device).synchronize()
        check(lib().nmx_nuts_init_from(ctypes.byref(self.cfg), ptr(self.arena), ptr(w), s))
        self._evaluate_all(s)
        check(lib().nmx_nuts_init_check(ctypes.byref(self.cfg), ptr(self.arena), s))
        bad = int(self.view("counters")[1].item())
        if bad:
            raise RuntimeError(f"{bad} chains have a non-finite potential after the mass-matrix update")

    def _positive(self):
        """Coordinates the collection maps through exp (ExpTransform sites), as a bool mask."""
        pos = self.model_potential.transform_codes().to(torch.bool)
        return pos if self.constrain_samples else torch.zeros_like(pos)

    def _collect_codes(self):
        """Transform codes the step kernels apply to collected draws (all zero: unconstrained)."""
        tr = self.potential.transform_codes()
        return tr if self.constrain_samples else torch.zeros_like(tr)

    def _convert_slots(self, samples, slots, s):
        """In place: whitened draws of collection slots -> model space -> constrained."""
        if len(slots) == 0 or samples.shape[0] == 0:
            return
        wt = self.potential.whitening
        tmp = torch.empty(self.D, self.ldc, dtype=torch.float32, device=self.device)
        pos = self._positive()
        for k in slots:
            wt.to_model(samples[k], tmp, stream=s)
            samples[k].copy_(tmp)
            if bool(pos.any()):
                samples[k][pos] = torch.exp(samples[k][pos])

    def _dense_segments(self, it0, it1):
        """Split [it0, it1) at the bounds of the middle adaptation windows; yields
        (a, b, window) with window = (start, end + 1) of the middle window holding [a, b), or
        None outside them."""
        bounds = []
        if self.opts.adapt_mass_matrix and self.num_warmup > 0:
            sched = build_adaptation_schedule(self.num_warmup)
            for i, (ws, we) in enumerate(sched):
                if 0 < i < len(sched) - 1:
                    bounds.append((ws, we + 1))
        segs, a = [], it0
        for ws, we1 in bounds:
            if we1 <= a or ws >= it1:
                continue
            if ws > a:
                segs.append((a, ws, None))
                a = ws
            b = min(we1, it1)
            segs.append((a, b, (ws, we1)))
            a = b
        if a < it1:
            segs.append((a, it1, None))
        return segs

    def run(self, num_iters: int, seed: int, collect_begin: int = 0, collection_size: int | None = None,
            thinning: int = 1, poll_every: int = 16, stream=None, max_launches: int | None = None,
            collect_samples: bool = True):
        """Advance every chain by `num_iters` transitions.  Transitions with relative index
        i >= start_idx (fori_collect semantics) are collected into the returned buffers.
        Returns (samples [S, D, ldc], fields [S, NC, ldc], launches); with collect_samples
        False only the fields are collected (samples is [0, D, ldc])."""
        s = stream_ptr(stream)
        num_iters = int(num_iters)
        lower = int(collect_begin)
        if collection_size is None:
            collection_size = (num_iters - lower) // thinning
        start_idx = lower + (num_iters - lower) % thinning  # util.py:330
        it0 = self.iteration
        if self.sync_chains and num_iters > self.iter_capacity:
            self._grow_finished(num_iters)
        S = max(int(collection_size), 0)
        if S > 0:
            samples = torch.empty((S if collect_samples else 0, self.D, self.ldc), dtype=torch.float32,
                                  device=self.device)
            fields = torch.zeros((S, len(native.COLLECT), self.ldc), dtype=torch.float32, device=self.device)
        else:  # nothing is collected: the device writes no slot (collection_size 0)
            samples = torch.empty((0, self.D, self.ldc), dtype=torch.float32, device=self.device)
            fields = torch.empty((0, len(native.COLLECT), self.ldc), dtype=torch.float32, device=self.device)
        self.generation = next(_generations)
        cstart = it0 + start_idx
        if not self.dense:
            # with the step-size search, stop at every middle-window end it runs at
            cuts = self._search_cuts(it0, it0 + num_iters)
            launches, a = 0, it0
            for b in sorted(set(cuts + [it0 + num_iters])):
                if b > a:
                    launches += self._run_segment(a, b, seed, cstart, thinning, S, samples, fields, poll_every, s,
                                                  max_launches)
                if b in cuts:
                    self._search_at_window_end(b, cstart, thinning, S, fields, s)
                a = b
        else:
            launches = self._run_dense(it0, it0 + num_iters, seed, cstart, thinning, S, samples, fields,
                                       poll_every, s, max_launches)
        self.iteration = it0 + num_iters
        self.generation = next(_generations)
        return samples, fields, launches

    @staticmethod
    def _slot_of(i, cstart, thinning, S):
        """Collection slot whose final value transition i writes (util.py:330-346: slot
        (i - start) // thinning, last write wins), or -1."""
        off = i - cstart
        if off < 0 or off % thinning != thinning - 1 or off // thinning >= S:
            return -1
        return off // thinning

    def _slots_in(self, a, b, cstart, thinning, S):
        """Collection slots completed by transitions [a, b)."""
        return [k for k in (self._slot_of(i, cstart, thinning, S) for i in range(a, b)) if k >= 0]

    def _run_dense(self, it0, it1, seed, cstart, thinning, S, samples, fields, poll_every, s, max_launches):
        """Dense mass: segments outside the middle windows run as they are; inside one, every
        transition's draws (model space) join the window's pool, which persists across run()
        calls (a kernel stepped one transition at a time pools the same draws), and the window's
        last transition finalizes it and re-expresses every chain."""
        from .dense import ChainWelford, PooledCovariance
        chunk = max(1, int(self.opts.dense_adapt_bytes) // (4 * self.D * self.ldc))
        wt = self.potential.whitening
        pos = self._positive()
        launches = 0
        for a, b, win in self._dense_segments(it0, it1):
            if win is None:
                # without mass adaptation the window ends still run the step-size search
                cuts = self._search_cuts(a, b)
                ends = sorted(set(cuts + [b]))
                for p, q in zip([a] + ends[:-1], ends):
                    if q > p:
                        launches += self._run_segment(p, q, seed, cstart, thinning, S, samples, fields, poll_every,
                                                      s, max_launches)
                        self._convert_slots(samples, self._slots_in(p, q, cstart, thinning, S), s)
                    if q in cuts:
                        self._search_at_window_end(q, cstart, thinning, S, fields, s)
                continue
            if self._pool is None or self._pool[0] != win:
                self._pool = (win, ChainWelford(self.D, self.C, self.device) if self.chain_dense
                              else PooledCovariance(self.D, self.device, wt.mu))
            pool = self._pool[1]
            zbuf = torch.empty(self.D, self.ldc, dtype=torch.float32, device=self.device)
            for ca in range(a, b, chunk):
                cb = min(b, ca + chunk)
                n = cb - ca
                abuf = torch.empty((n, self.D, self.ldc), dtype=torch.float32, device=self.device)
                afld = torch.zeros((n, len(native.COLLECT), self.ldc), dtype=torch.float32, device=self.device)
                launches += self._run_segment(ca, cb, seed, ca, 1, n, abuf, afld, poll_every, s, max_launches)
                for k in range(n):
                    wt.to_model(abuf[k], zbuf, stream=s)
                    if self.chain_dense:
                        pool.add(zbuf, stream=s)
                    else:
                        pool.add(zbuf[:, :self.C])
                    slot = self._slot_of(ca + k, cstart, thinning, S)
                    if slot >= 0:
                        if samples.shape[0] > 0:
                            samples[slot].copy_(zbuf)
                            if bool(pos.any()):
                                samples[slot][pos] = torch.exp(samples[slot][pos])
                        fields[slot].copy_(afld[k])
                del abuf, afld
            if b == win[1]:
                if self.chain_dense:
                    cov, mean = pool.finalize(self.opts.regularize_mass_matrix, self.blocks), None
                else:
                    pool.all_reduce(self.device_group)
                    cov, mean = pool.finalize(self.opts.regularize_mass_matrix)
                self._pool = None
                self._reexpress(cov, mean, s)
                if self._heuristic():
                    self._search_at_window_end(b, cstart, thinning, S, fields, s)
        return launches

    def _persistent_model(self):
        """(model id, p0, p1, n) when the run can use the one-launch persistent schedule
        (nmx_nuts_run_small: one-wave model with an inline potential, per-chain async)."""
        if self.sync_chains or self.D >= 16 or not self.persistent:
            return None
        fn = getattr(self.potential, "small_model", None)
        return fn() if fn is not None else None

    def _wide_model(self):
        """(model id, data, n) when the step can run fused with a D-split model's potential
        (nmx_nuts_step_wide_model: three launches per leaf instead of six)."""
        if self.dense or not self.fused_wide or lib().nmx_nuts_num_slices(self.D) == 0:
            return None
        fn = getattr(self.potential, "wide_model", None)
        return fn() if fn is not None else None

    def _run_segment(self, a, b, seed, cstart, thinning, S, samples, fields, poll_every, s, max_launches):
        """Transitions [a, b) of every chain; collection slots per (cstart, thinning, S)."""
        self._fill_cfg(a, b, self.num_warmup, seed, cstart, thinning, S)
        cfgp = ctypes.byref(self.cfg)
        arena = ptr(self.arena)
        tr = self._collect_codes()
        if self.persist_wide:
            return self._run_wide_persistent(a, b, seed, cstart, thinning, S, samples, fields, s, max_launches)
        check(lib().nmx_nuts_resume(cfgp, arena, s), "nmx_nuts_resume")
        small = self._persistent_model()
        if small is not None:
            # one launch normally covers the segment (NUTS: <= 2^depth + 2 steps per
            # transition); HMC trajectories (ceil(L / step) leapfrogs) may need more: the
            # kernel resumes from the arena, so relaunch until every chain is DONE
            model, p0, p1, n = small
            max_steps = (b - a) * ((1 << self.md) + 2) + 16
            launches = 0
            while True:
                check(lib().nmx_nuts_run_small(cfgp, arena, ptr(samples) if samples.shape[0] else None, ptr(fields),
                                               ptr(tr), model, ptr(p0),
                                               ptr(p1), n, max_steps, s), "nmx_nuts_run_small")
                launches += 1
                if int(self.view("counters")[0].item()) >= self.C:
                    return launches
                if max_launches is not None and launches * max_steps >= max_launches:
                    raise RuntimeError(f"chains did not finish within {max_launches} leapfrog steps")
        groups = self._groups()
        if groups > 1:
            return self._run_groups(groups, samples, fields, tr, poll_every, s, max_launches)
        done = self.view("counters")[0:1]
        host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        ev = torch.cuda.Event()
        pending = False
        launches = 0
        step = lib().nmx_nuts_step
        sp, fp, tp = ptr(samples) if samples.shape[0] else None, ptr(fields), ptr(tr)
        cfg = self.cfg
        parity = 0
        cfg.parity = parity
        check(step(cfgp, arena, sp, fp, tp, s), "nmx_nuts_step")
        evaluate = self.potential.evaluate
        lists = self.eval_lists
        for b in lists:
            b.num_chains = self.C
        wide = self._wide_model()
        if wide is not None:
            model, data, n = wide
            if self._wide_ws is None:
                nb = lib().nmx_nuts_wide_model_workspace_bytes(self.D, self.C)
                self._wide_ws = torch.zeros(nb, dtype=torch.uint8, device=self.device)
            wstep, dp, wsp = lib().nmx_nuts_step_wide_model, ptr(data), ptr(self._wide_ws)
        while True:
            for _ in range(poll_every):
                if wide is not None:
                    check(wstep(cfgp, arena, sp, fp, tp, model, dp, n, wsp, s), "nmx_nuts_step_wide_model")
                    continue
                evaluate(lists[parity], s)
                parity ^= 1
                cfg.parity = parity
                check(step(cfgp, arena, sp, fp, tp, s), "nmx_nuts_step")
            launches += poll_every
            if pending:
                ev.synchronize()
                done_n = int(host[0])
                if done_n >= self.C:
                    break
                # finished chains never re-enter the lists: C - done bounds every later list
                # count, and kernels size their grids by it (nmx_eval_batch.num_chains)
                for b in lists:
                    b.num_chains = self.C - done_n
            host.copy_(done, non_blocking=True)
            ev.record()
            pending = True
            if max_launches is not None and launches >= max_launches:
                raise RuntimeError(f"chains did not finish within {max_launches} leapfrog launches")
        return launches

    def _groups(self):
        """Chain groups of the launched fused step (1: none): dim <= 256 models whose potential
        keeps a workspace per concurrently evaluated group, at >= 128 chains per group.  Also
        under the lockstep schedule (sync_chains): a waiting chain's release is decided once per
        chain inside the step (nuts.hip wait_released), so other streams' writes to the
        transition counts only decide WHEN a chain starts, never what it computes."""
        G = int(self.chain_groups)
        if G <= 1 or self.dense or self.crow or lib().nmx_nuts_num_slices(self.D) > 0:
            return 1
        if getattr(self.potential, "slots", 1) < G or self.C < 128 * G:
            return 1
        return G

    def _run_groups(self, G, samples, fields, tr, poll_every, s, max_launches):
        """The launched loop with chain groups (nmx_nuts_config.num_groups): group g's potential
        and step launches go to stream g (the caller's stream for g = 0), each group with its
        own compacted lists and DONE count, so a group's latency-bound step, finalize and run
        tail overlap the other groups' potential.  A chain's computation does not depend on its
        group: draws are bitwise those of the one-stream loop."""
        main = torch.cuda.ExternalStream(s, device=self.device)
        while len(self._side_streams) < G - 1:
            self._side_streams.append(torch.cuda.Stream(device=self.device))
        streams = [main] + self._side_streams[:G - 1]
        raw = [s] + [int(st.cuda_stream) for st in streams[1:]]
        start = torch.cuda.Event()
        start.record(main)
        for st in streams[1:]:
            st.wait_event(start)  # after the resume / setup issued on the caller's stream
        gsz = (self.C + G - 1) // G
        sizes = [max(0, min(gsz, self.C - g * gsz)) for g in range(G)]
        step = lib().nmx_nuts_step
        arena = ptr(self.arena)
        sp, fp, tp = ptr(samples) if samples.shape[0] else None, ptr(fields), ptr(tr)
        idx, cnt = ptr(self.view("active_idx")), ptr(self.view("counters"))
        z, gr, pe, ph = (ptr(self.view(n)) for n in ("z_eval", "g_eval", "pe_eval", "phase"))
        counters = self.view("counters")
        cfgs, lists, par = [], [], [0] * G
        for g in range(G):
            c = NutsConfig.from_buffer_copy(self.cfg)
            c.num_groups, c.group, c.parity = G, g, 0
            cfgs.append(c)
            lists.append([EvalBatch(z=z, grad=gr, pe=pe, phase=ph, active_idx=idx + 4 * (p * self.ldc + g * gsz),
                                    active_count=cnt + 4 * (2 + 2 * g + p), num_chains=max(sizes[g], 1),
                                    ldc=self.ldc) for p in (0, 1)])
            check(step(ctypes.byref(c), arena, sp, fp, tp, raw[g]), "nmx_nuts_step")
        evaluate = self.potential.evaluate
        hosts = [torch.zeros(1, dtype=torch.int32, pin_memory=True) for _ in range(G)]
        evs = [torch.cuda.Event() for _ in range(G)]
        pending, live = [False] * G, [sizes[g] > 0 for g in range(G)]
        launches = 0
        while any(live):
            for _ in range(poll_every):
                for g in range(G):
                    if not live[g]:
                        continue
                    evaluate(lists[g][par[g]], raw[g], g)
                    par[g] ^= 1
                    cfgs[g].parity = par[g]
                    check(step(ctypes.byref(cfgs[g]), arena, sp, fp, tp, raw[g]), "nmx_nuts_step")
            launches += poll_every
            for g in range(G):
                if not live[g]:
                    continue
                if pending[g]:
                    evs[g].synchronize()
                    done_g = int(hosts[g][0])
                    if done_g >= sizes[g]:
                        live[g] = False
                        continue
                    for b in lists[g]:  # finished chains never re-enter the group's lists
                        b.num_chains = sizes[g] - done_g
                with torch.cuda.stream(streams[g]):
                    hosts[g].copy_(counters[10 + g:11 + g], non_blocking=True)
                    evs[g].record(streams[g])
                pending[g] = True
            if max_launches is not None and launches >= max_launches:
                raise RuntimeError(f"chains did not finish within {max_launches} leapfrog launches")
        for st in streams[1:]:  # the caller's stream continues after every group's work
            j = torch.cuda.Event()
            j.record(st)
            main.wait_event(j)
        return launches

    def _run_wide_persistent(self, a, b, seed, cstart, thinning, S, samples, fields, s, max_launches):
        """nmx_nuts_run_wide: one launch runs every chain through [a, b) (relaunched while
        some chain hit the leaf bound, e.g. long HMC trajectories).  The lockstep schedule
        (sync_chains) is one launch per transition: no chain starts transition t + 1 before
        every chain finished t, and each chain's computation is the same as unsynchronised."""
        model, data, n = self.potential.wide_model()
        tr = self._collect_codes()
        sp, fp, tp, dp = ptr(samples) if samples.shape[0] else None, ptr(fields), ptr(tr), ptr(data)
        run = lib().nmx_nuts_run_wide
        spans = [(t, t + 1) for t in range(a, b)] if self.sync_chains else [(a, b)]
        launches = 0
        for t0, t1 in spans:
            self._fill_cfg(t0, t1, self.num_warmup, seed, cstart, thinning, S)
            self.cfg.sync_chains = 0
            cfgp = ctypes.byref(self.cfg)
            check(lib().nmx_nuts_resume(cfgp, ptr(self.arena), s), "nmx_nuts_resume")
            max_steps = (t1 - t0) * ((1 << self.md) + 2) + 16
            while True:
                check(run(cfgp, ptr(self.arena), sp, fp, tp, model, dp, n, max_steps, s), "nmx_nuts_run_wide")
                launches += 1
                if int(self.view("counters")[0].item()) >= self.C:
                    break
                if max_launches is not None and launches * max_steps >= max_launches:
                    raise RuntimeError(f"chains did not finish within {max_launches} leapfrog steps")
        return launches

    def _grow_finished(self, n):
        # re-layout the arena with a larger sync-counter table, keeping all chain state
        old = self.arena
        old_views = {k: self.view(k).clone() for k in native.FIELDS if k != "finished"}
        self._alloc(n)
        for k, v in old_views.items():
            self.view(k).copy_(v)
        del old

    # ------------------------------------------------------------------ accessors
    def model_gradient(self, z):
        """grad U at model-space unconstrained positions z [D, ldc] (every chain < C): the model's
        own potential kernel on a dense batch, as during sampling (MCMC's z_grad extra field)."""
        g = torch.zeros_like(z)
        pe = torch.zeros(self.ldc, dtype=torch.float32, device=self.device)
        ev = EvalBatch(z=ptr(z), grad=ptr(g), pe=ptr(pe), phase=None, active_idx=None, active_count=None,
                       num_chains=self.C, ldc=self.ldc)
        self.model_potential.evaluate(ev, stream_ptr())
        return g

    def model_state(self):
        """(z [C, D], grad U(z) [C, D]) in model coordinates (un-whitened for dense mass)."""
        z, g = self.chain_state("z"), self.chain_state("zgrad")
        if not self.dense:
            return z.clone(), g.clone()
        wt = self.potential.whitening
        zb = torch.empty(self.D, self.ldc, dtype=torch.float32, device=self.device)
        wt.to_model(self.view("z").contiguous(), zb, stream=stream_ptr())
        # g_w = T^T g_z  ->  g_z = T^-T g_w
        return zb[:, :self.C].t().clone(), wt.grad_to_model(g.t()).t().contiguous()

    def mass_state(self):
        """(inverse_mass_matrix, mass_matrix_sqrt, mass_matrix_sqrt_inv) as HMCAdaptState holds
        them: per-chain diagonals [C, D], per-chain dense matrices [C, D, D], or the pooled /
        shared dense matrices [D, D]."""
        if self.dense:
            # the matrices change only when the whitening is set (window ends): computed once
            # per version (mass_matrix_sqrt is a triangular solve) and shared by every snapshot
            # until then; Whitening.set replaces them, never writes into them
            wt = self.potential.whitening
            key = (id(wt), wt.version)
            if self._mass_cache is None or self._mass_cache[0] != key:
                mats = (wt.inverse_mass_matrix.to(torch.float32), wt.mass_matrix_sqrt().to(torch.float32),
                        wt.mass_matrix_sqrt_inv().to(torch.float32).clone())
                if self.blocks is not None:  # {site group: block} dicts, as HMCAdaptState holds them
                    mats = tuple(self.blocks.split(m) if self.chain_dense else
                                 {k: v[0] for k, v in self.blocks.split(m[None]).items()} for m in mats)
                self._mass_cache = (key, mats)
            return self._mass_cache[1]
        ms = self.chain_state("mass_sqrt").clone()
        return self.chain_state("inv_mass").clone(), ms, 1.0 / ms

    def whitening_state(self):
        if not self.dense:
            return None
        wt = self.potential.whitening
        # inverse_mass_matrix is replaced by Whitening.set, not written: shared; mu is written
        return (wt.inverse_mass_matrix, None if self.chain_dense else wt.mu.clone())

    def set_whitening_state(self, st):
        if st is not None:
            self.potential.whitening.set(st[0], st[1])

    def layout(self):
        """What a state's arena copy must match to be resumed by this engine (a pickled
        state is resumed by the engine of an unpickled MCMC / kernel in another process)."""
        return (type(self.model_potential).__name__, self.C, self.D, self.md, self.chain_offset, self.dense,
                self.chain_dense, self.opts.algo, self.crow)

    def chain_state(self, name):
        """Per-chain view without padding: scalars [C], vectors [C, D]."""
        v = self.view(name)
        if v.dim() == 1:
            return v[:self.C]
        return v[:, :self.C].t()
