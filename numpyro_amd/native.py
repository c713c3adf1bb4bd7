"""ctypes binding of the C-ABI in ``include/numpyro_amd.h``.

``torch`` is imported first on purpose: torch-ROCm ships its own ``libamdhip64.so.7``;
loading it before our library makes the dynamic linker resolve our ``DT_NEEDED``
``libamdhip64.so.7`` to that same copy, so the ``hipStream_t`` handles torch gives us
belong to the runtime our kernels launch through.

The product path never falls back: if the library is missing this raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# NUMPYRO_AMD_DEBUG=1: the debug build (bounds / invariant checks, numpyro_amd.build(debug=True))
LIB_PATH = os.path.join(_HERE, "_lib", "libnumpyro_amd_debug.so" if os.environ.get("NUMPYRO_AMD_DEBUG") == "1"
                        else "libnumpyro_amd.so")
# kernel experiments: another in-tree build of the same library (scripts/ab_build.py variants)
if os.environ.get("NUMPYRO_AMD_LIB"):
    LIB_PATH = os.path.abspath(os.environ["NUMPYRO_AMD_LIB"])

_lib = None

c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_size = ctypes.c_size_t
c_float = ctypes.c_float
c_double = ctypes.c_double
c_vp = ctypes.c_void_p

MAX_WINDOWS = 32  # NMX_MAX_WINDOWS
MAX_TREE_DEPTH = 12  # NMX_MAX_TREE_DEPTH

ALGO_NUTS, ALGO_HMC = 0, 1
PH_DONE, PH_WAIT, PH_START, PH_LEAF, PH_INITEVAL, PH_NEEDINIT = range(6)

# enum nmx_field (order matters)
FIELDS = [
    "phase", "iter", "depth", "sub_n", "dir", "tree_n", "window_idx", "da_t", "wf_n", "turning",
    "tree_div", "sub_div", "hmc_k", "hmc_n", "last_nsteps", "last_div", "maxdepth_cur",
    "hs_k", "hs_dir", "hs_last",
    "action", "slot", "act_wfn",
    "step_size", "e0", "pe", "energy", "tree_w", "tree_acc", "sub_w", "sub_acc", "pe_sub", "e_sub",
    "da_xt", "da_xavg", "da_gavg", "da_prox", "mean_acc", "last_acc", "step_eff", "hs_step",
    "hs_e0", "pe_eval",
    "z", "zgrad", "zl", "rl", "gl", "zr", "rr", "gr", "zsub", "gsub", "rsum", "rsum_sub",
    "inv_mass", "mass_sqrt", "wf_mean", "wf_m2", "z_eval", "g_eval",
    "ckpt_r", "ckpt_rsum", "active_idx", "counters", "finished", "part", "part0", "tot",
]
FIELD_ID = {n: i for i, n in enumerate(FIELDS)}
INT_FIELDS = set(FIELDS[:FIELDS.index("step_size")]) | {"counters", "finished", "active_idx"}
VECTOR_FIELDS = set(FIELDS[FIELDS.index("z"):FIELDS.index("ckpt_r")])
CKPT_FIELDS = {"ckpt_r", "ckpt_rsum"}

# enum nmx_collect
COLLECT = ["potential_energy", "energy", "accept_prob", "mean_accept_prob", "step_size",
           "num_steps", "diverging", "i"]


class NutsConfig(ctypes.Structure):
    """Mirror of nmx_nuts_config (include/numpyro_amd.h)."""

    _fields_ = [
        ("algo", ctypes.c_int32), ("num_chains", ctypes.c_int32), ("dim", ctypes.c_int32),
        ("max_depth_alloc", ctypes.c_int32), ("max_tree_depth_warmup", ctypes.c_int32),
        ("max_tree_depth", ctypes.c_int32), ("num_warmup", ctypes.c_int32),
        ("iter_end", ctypes.c_int32), ("iter_begin", ctypes.c_int32),
        ("iter_capacity", ctypes.c_int32), ("adapt_step_size", ctypes.c_int32),
        ("adapt_mass_matrix", ctypes.c_int32), ("regularize_mass_matrix", ctypes.c_int32),
        ("unit_mass", ctypes.c_int32), ("sync_chains", ctypes.c_int32),
        ("target_accept_prob", ctypes.c_float), ("max_delta_energy", ctypes.c_float),
        ("trajectory_length", ctypes.c_float), ("num_steps", ctypes.c_int32),
        ("num_windows", ctypes.c_int32), ("window_end", ctypes.c_int32 * MAX_WINDOWS),
        ("seed", ctypes.c_uint64), ("chain_offset", ctypes.c_int64),
        ("collect_start", ctypes.c_int32), ("collect_thinning", ctypes.c_int32),
        ("collection_size", ctypes.c_int32), ("ldc", ctypes.c_int32), ("parity", ctypes.c_int32),
        ("layout", ctypes.c_int32), ("num_groups", ctypes.c_int32), ("group", ctypes.c_int32),
        ("trace_chains", ctypes.c_int32), ("trace_it0", ctypes.c_int32), ("trace_iters", ctypes.c_int32),
        ("trace_leaves", ctypes.c_int32), ("trace", c_vp),
    ]


# per-leaf decision trace (nmx_nuts_config.trace): record layout and flag bits
TRACE_REC = 8  # NMX_TRACE_REC
TRACE_FIELDS = ["dE", "p_leaf", "dot_sub", "p_biased", "dot_tree", "flags", "pe", "leaf"]  # enum nmx_trace_field
TF_TAKE_LEAF, TF_TURN_SUB, TF_DIVERGE, TF_DONE_SUB, TF_TAKE_BIASED, TF_TURN_TREE, TF_ITER_DONE = (
    1, 2, 4, 8, 16, 32, 64)  # enum nmx_trace_flag


LAYOUT_CHAIN_MINOR, LAYOUT_CHAIN_ROWS = 0, 1  # enum nmx_layout


SMALL_DIAG_NORMAL, SMALL_EIGHT_SCHOOLS = 1, 2  # nmx_nuts_run_small models
WIDE_SV, WIDE_FUNNEL, WIDE_FUNNEL_NC = 1, 2, 3  # nmx_nuts_step_wide_model models


class EvalBatch(ctypes.Structure):
    """Mirror of nmx_eval_batch."""

    _fields_ = [("z", c_vp), ("grad", c_vp), ("pe", c_vp), ("phase", c_vp),
                ("active_idx", c_vp), ("active_count", c_vp),
                ("num_chains", ctypes.c_int32), ("ldc", ctypes.c_int32)]


_P = ctypes.POINTER
_cfgp = _P(NutsConfig)
_evp = _P(EvalBatch)

# name -> (restype, argtypes); kept in sync with include/numpyro_amd.h (tests check it).
SIGNATURES: dict[str, tuple] = {
    "nmx_version": (c_int, []),
    "nmx_last_error": (ctypes.c_char_p, []),
    "nmx_struct_size": (c_size, [c_int]),
    "nmx_selftest_philox": (c_int, [c_vp, c_vp, c_int, c_vp]),
    "nmx_selftest_mfma": (c_int, [c_vp, c_vp, c_vp, c_int, c_vp]),
    "nmx_selftest_dcheck": (c_int, [c_int, c_vp]),
    "nmx_selftest_expf": (c_int, [c_vp, c_vp, c_vp, c_int, c_vp]),
    "nmx_nuts_arena_bytes": (c_size, [c_int, c_int, c_int, c_int]),
    "nmx_nuts_num_slices": (c_int, [c_int]),
    "nmx_nuts_field_info": (c_int, [c_int, c_int, c_int, c_int, c_int, _P(c_size), _P(c_size)]),
    "nmx_nuts_reset": (c_int, [_cfgp, c_vp, c_float, c_vp, c_vp]),
    "nmx_nuts_init_draw": (c_int, [_cfgp, c_vp, c_int, c_float, c_vp]),
    "nmx_nuts_init_from": (c_int, [_cfgp, c_vp, c_vp, c_vp]),
    "nmx_nuts_init_check": (c_int, [_cfgp, c_vp, c_vp]),
    "nmx_nuts_resume": (c_int, [_cfgp, c_vp, c_vp]),
    "nmx_heuristic_begin": (c_int, [_cfgp, c_vp, c_vp]),
    "nmx_heuristic_propose": (c_int, [_cfgp, c_vp, c_vp]),
    "nmx_heuristic_finish": (c_int, [_cfgp, c_vp, c_int, c_vp]),
    "nmx_heuristic_noise": (c_int, [_cfgp, c_vp, c_vp, c_vp]),
    "nmx_heuristic_propose_with": (c_int, [_cfgp, c_vp, c_vp, c_vp]),
    "nmx_nuts_run_small": (c_int, [_cfgp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_int, c_vp]),
    "nmx_nuts_run_wide": (c_int, [_cfgp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_vp]),
    "nmx_predict_logreg": (c_int, [c_vp, ctypes.c_int64, c_int, c_vp, c_int, ctypes.c_uint64, c_vp, c_vp]),
    "nmx_predict_normal": (c_int, [c_vp, c_vp, c_int, c_int, ctypes.c_uint64, c_vp, c_vp]),
    "nmx_predict_bnn": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, ctypes.c_uint64, c_vp, c_vp]),
    "nmx_nuts_step": (c_int, [_cfgp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "nmx_nuts_wide_model_workspace_bytes": (c_size, [c_int, c_int]),
    "nmx_nuts_step_wide_model": (c_int, [_cfgp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp, c_vp]),
    "nmx_pe_diag_normal": (c_int, [c_vp, c_vp, c_int, _evp, c_vp]),
    "nmx_pe_eight_schools": (c_int, [c_vp, c_vp, c_int, _evp, c_vp]),
    "nmx_pe_stochastic_volatility": (c_int, [c_vp, c_int, _evp, c_vp, c_vp]),
    "nmx_pe_funnel": (c_int, [c_int, _evp, c_vp, c_vp]),
    "nmx_pe_funnel_noncentered": (c_int, [c_int, _evp, c_vp, c_vp]),
    "nmx_pe_wide_workspace_bytes": (c_size, [c_int, c_int]),
    "nmx_pe_bnn": (c_int, [c_vp, c_vp, c_int, c_int, c_int, _evp, c_vp, c_vp]),
    "nmx_pe_bnn_workspace_bytes": (c_size, [c_int, c_int, c_int]),
    "nmx_pe_bnn_rows": (c_int, [c_vp, c_vp, c_int, c_int, c_int, _evp, c_vp, c_vp, c_vp]),
    "nmx_logreg_packed_bytes": (c_size, [c_i64, c_int]),
    "nmx_logreg_pack": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_vp]),
    "nmx_logreg_workspace_bytes": (c_size, [c_i64, c_int, c_int]),
    "nmx_logreg_pe_grad": (c_int, [c_vp, c_i64, c_int, _evp, c_vp, c_vp]),
    "nmx_logreg_num_splits": (c_int, [c_i64]),
    "nmx_dense_padded_dim": (c_int, [c_int]),
    "nmx_gemm_chains": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp]),
    "nmx_gemm_chains_workspace_bytes": (c_size, [c_int, c_int]),
    "nmx_gemm_x3_packed_a_bytes": (c_size, [c_int]),
    "nmx_gemm_x3_pack_a": (c_int, [c_vp, c_int, c_vp, c_vp]),
    "nmx_gemm_x3_split_bytes": (c_size, [c_int, c_int]),
    "nmx_gemm_chains_x3": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp,
                                   c_vp]),
    "nmx_gemm_chains_x3_rows": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_int, c_vp,
                                        c_vp, c_vp]),
    "nmx_gemm_chains_x3_to_rows": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_int,
                                           c_vp, c_vp, c_vp, c_vp]),
    "nmx_gemm_chains_x3_lists": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp,
                                         c_int, c_vp, c_vp, c_vp, c_vp]),
    "nmx_pack_columns": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp]),
    "nmx_chain_matvec": (c_int, [c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_vp]),
    "nmx_chain_welford": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    "nmx_chain_matvec_tri": (c_int, [c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_vp]),
    "nmx_chain_welford_work_bytes": (c_size, [c_int, c_int]),
    "nmx_chain_welford_ws": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "nmx_unpack_columns": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp]),
    "nmx_pack_rows": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp]),
    "nmx_unpack_rows": (c_int, [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp]),
    "nmx_pe_mvn": (c_int, [c_vp, c_int, c_vp, c_vp, c_int, _evp, c_vp]),
}


class NativeError(RuntimeError):
    pass


def lib():
    """Load (once) and return the ctypes handle; raises if the library is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"numpyro_amd native library not found at {LIB_PATH}; "
                "run `python -m numpyro_amd.build` (or __graft_entry__.build())"
            )
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = lib().nmx_last_error().decode(errors="replace")
        raise NativeError(f"{what or 'numpyro_amd'} failed (status {status}): {msg}")


def stream_ptr(stream=None) -> int:
    """Raw hipStream_t of a torch stream (the current stream by default)."""
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)


def ptr(t) -> int:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return 0
    return int(t.data_ptr())
