/*
 * numpyro_amd C-ABI: the drop-in boundary of the MI355X-native NUTS/HMC engine.
 *
 * The reference (fehiepsi/numpyro) has no native code: its hot path is Python traced by
 * JAX/XLA.  Each entry point below replaces one piece of that traced path; the comment
 * on each names the reference function (file:line under numpyro/) it stands in for.
 * INTEGRATION.md shows the ctypes binding a numpyro maintainer would add.
 *
 * Conventions
 *  - extern "C", plain pointers and sizes; no torch types.  All pointers are device
 *    pointers unless named host_*.  `stream` is a hipStream_t passed as void*.
 *  - Chain-major SoA: a per-chain vector field is stored [D][ldc] (ldc >= C, ldc % 64 == 0),
 *    so lanes of a wave read consecutive chains.  Per-chain scalars are [ldc].  The arena of
 *    the persistent wide schedule (nmx_nuts_run_wide) instead stores vector fields in chain
 *    rows [ldc][D] (cfg->layout = NMX_LAYOUT_CHAIN_ROWS): one workgroup per chain reads the
 *    chain's contiguous row.  Buffers passed in and out (init z, samples) are [D][ldc] always.
 *  - The library never allocates on the hot path: callers allocate the arena / workspace
 *    whose size the *_bytes() queries return.
 *  - Return value: NMX_OK or an error code; nmx_last_error() has the message.  Numerical
 *    events (divergence, NaN energy) are data, never errors (hmc_util.py:870-874).
 */
#ifndef NUMPYRO_AMD_H
#define NUMPYRO_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NMX_VERSION 1

enum nmx_status {
  NMX_OK = 0,
  NMX_ERR_INVALID = 1,     /* API misuse: bad size, null pointer, unsupported combo */
  NMX_ERR_HIP = 2,         /* HIP runtime error (launch failure etc.) */
  NMX_ERR_UNSUPPORTED = 3, /* configuration not implemented */
};

int nmx_version(void);
const char* nmx_last_error(void);
/* sizeof of the ABI structs (0: nmx_nuts_config, 1: nmx_eval_batch), for binding checks. */
size_t nmx_struct_size(int which);

/* ======================================================================================
 * Vectorized-chain NUTS / HMC engine (numpyro/infer/hmc.py + numpyro/infer/hmc_util.py)
 * ====================================================================================== */

#define NMX_MAX_WINDOWS 32
#define NMX_MAX_TREE_DEPTH 12

enum nmx_algo { NMX_ALGO_NUTS = 0, NMX_ALGO_HMC = 1 };

/* Per-chain phase codes stored in the arena's `phase` field. */
enum nmx_phase {
  NMX_PH_DONE = 0,      /* finished iter_end transitions */
  NMX_PH_WAIT = 1,      /* sync_chains: waiting for the other chains of this device */
  NMX_PH_START = 2,     /* will start a new transition at the next nmx_nuts_step */
  NMX_PH_LEAF = 3,      /* a leapfrog is pending: potential(z_eval) must be evaluated */
  NMX_PH_INITEVAL = 4,  /* initial point pending evaluation */
  NMX_PH_NEEDINIT = 5,  /* no valid initial point yet */
};
/* Potential kernels evaluate chains whose phase >= NMX_PH_LEAF. */

/* Arena fields (SoA). Vector fields are [D][ldc] float; ckpt fields [max_depth][D][ldc]
 * ([ldc][D] and [max_depth][ldc][D] in the NMX_LAYOUT_CHAIN_ROWS layout; same sizes). */
enum nmx_layout { NMX_LAYOUT_CHAIN_MINOR = 0, NMX_LAYOUT_CHAIN_ROWS = 1 };
enum nmx_field {
  /* per-chain int32 scalars */
  NMX_F_PHASE = 0, NMX_F_ITER, NMX_F_DEPTH, NMX_F_SUB_N, NMX_F_DIR, NMX_F_TREE_N,
  NMX_F_WINDOW_IDX, NMX_F_DA_T, NMX_F_WF_N, NMX_F_TURNING, NMX_F_TREE_DIV, NMX_F_SUB_DIV,
  NMX_F_HMC_K, NMX_F_HMC_N, NMX_F_LAST_NSTEPS, NMX_F_LAST_DIV, NMX_F_MAXDEPTH_CUR,
  NMX_F_HS_K, NMX_F_HS_DIR, NMX_F_HS_LAST,
  /* decisions of the last step, consumed by the wide (D-split) vector kernels */
  NMX_F_ACTION, NMX_F_SLOT, NMX_F_ACT_WFN,
  /* per-chain float scalars */
  NMX_F_STEP_SIZE, NMX_F_E0, NMX_F_PE, NMX_F_ENERGY, NMX_F_TREE_W, NMX_F_TREE_ACC,
  NMX_F_SUB_W, NMX_F_SUB_ACC, NMX_F_PE_SUB, NMX_F_E_SUB, NMX_F_DA_XT, NMX_F_DA_XAVG,
  NMX_F_DA_GAVG, NMX_F_DA_PROX, NMX_F_MEAN_ACC, NMX_F_LAST_ACC, NMX_F_STEP_EFF, NMX_F_HS_STEP,
  NMX_F_HS_E0, NMX_F_PE_EVAL,
  /* per-chain vectors [D][ldc] */
  NMX_F_Z, NMX_F_ZGRAD, NMX_F_ZL, NMX_F_RL, NMX_F_GL, NMX_F_ZR, NMX_F_RR, NMX_F_GR,
  NMX_F_ZSUB, NMX_F_GSUB, NMX_F_RSUM, NMX_F_RSUM_SUB, NMX_F_INV_MASS, NMX_F_MASS_SQRT,
  NMX_F_WF_MEAN, NMX_F_WF_M2, NMX_F_Z_EVAL, NMX_F_G_EVAL,
  /* checkpoints [max_depth][D][ldc] */
  NMX_F_CKPT_R, NMX_F_CKPT_RSUM,
  /* compacted list of LEAF chains for the next potential launch, int32 [2][ldc] by parity */
  NMX_F_ACTIVE_IDX,
  /* device counters int32[16]: [0] chains DONE, [1] chains NEEDINIT, [2 + 2 g + parity]
   * active-list lengths of chain group g (nmx_nuts_config.num_groups), [10 + g] chains of
   * group g DONE (num_groups > 1), [14..] reserved */
  NMX_F_COUNTERS,
  /* sync_chains: int32[iter_capacity] #chains that finished transition iter_begin + i */
  NMX_F_FINISHED,
  /* wide (D-split) step only: per-slice partial dot products f32 [NS][2*MAXD+2][ldc] and
   * momentum kinetic-energy partials [NS][ldc]; NS = nmx_nuts_num_slices(dim) (0: fused) */
  NMX_F_PART, NMX_F_PART0,
  /* wide step only: slice-reduced totals f32 [2*MAXD+3 + 1][ldc] */
  NMX_F_TOT,
  NMX_NUM_FIELDS
};

/* Collected per-sample scalar fields, layout fields[slot][NMX_NUM_COLLECT][ldc] float. */
enum nmx_collect {
  NMX_C_POTENTIAL_ENERGY = 0, NMX_C_ENERGY, NMX_C_ACCEPT_PROB, NMX_C_MEAN_ACCEPT_PROB,
  NMX_C_STEP_SIZE, NMX_C_NUM_STEPS, NMX_C_DIVERGING, NMX_C_ITER, NMX_NUM_COLLECT
};

typedef struct nmx_nuts_config {
  int32_t algo;                  /* nmx_algo */
  int32_t num_chains;            /* chains on this device (C) */
  int32_t dim;                   /* flattened latent size (D) */
  int32_t max_depth_alloc;       /* checkpoint rows allocated (>= both depths below) */
  int32_t max_tree_depth_warmup; /* hmc.py:299-303 (d1, d2) */
  int32_t max_tree_depth;
  int32_t num_warmup;            /* adaptation steps, hmc.py:297 */
  int32_t iter_end;              /* a chain is DONE after this many transitions */
  int32_t iter_begin;            /* first transition index of this run (sync counters) */
  int32_t iter_capacity;         /* rows of NMX_F_FINISHED (>= iter_end - iter_begin) */
  int32_t adapt_step_size;       /* hmc_util.py:518-707 flags */
  int32_t adapt_mass_matrix;
  int32_t regularize_mass_matrix;
  int32_t unit_mass;             /* 1: the inverse mass matrix is the identity for every chain
                                    and is not adapted (dense mass runs as identity mass on
                                    whitened coordinates around the potential, nmx_gemm_chains;
                                    or no adaptation and no user matrix): the step skips the
                                    inv_mass / mass_sqrt loads */
  int32_t sync_chains;           /* 1: reference vmap lockstep per transition */
  float target_accept_prob;
  float max_delta_energy;        /* hmc.py:188 */
  float trajectory_length;       /* HMC; <= 0 means None */
  int32_t num_steps;             /* HMC fixed steps; 0 means None */
  int32_t num_windows;           /* build_adaptation_schedule(num_warmup), hmc_util.py:387 */
  int32_t window_end[NMX_MAX_WINDOWS];
  uint64_t seed;                 /* Philox key */
  int64_t chain_offset;          /* global id of chain 0 on this device */
  int32_t collect_start;         /* fori_collect start_idx (util.py:330) */
  int32_t collect_thinning;
  int32_t collection_size;       /* slots in samples/fields; 0 disables collection */
  int32_t ldc;                   /* round_up(C, 64) */
  int32_t parity;                /* launch parity: nmx_nuts_step appends LEAF chains to
                                    active list [parity] (and clears [parity ^ 1]) */
  int32_t layout;                /* nmx_layout of the arena's vector fields: CHAIN_MINOR for
                                    every entry point but nmx_nuts_run_wide, which needs
                                    CHAIN_ROWS (reset / init / resume take either) */
  int32_t num_groups;            /* chain groups of the launched fused step (dim <= 256), 0/1:
                                    one group.  Group g holds chains [g G, min((g + 1) G, C)),
                                    G = ceil(C / num_groups), num_groups in {1, 2, 4}; each
                                    group has its own pair of compacted lists (entries
                                    [g G, ...) of each parity list, lengths counters[2 + 2 g +
                                    parity]), so groups step and evaluate independently, e.g.
                                    on two streams that overlap one group's step with the
                                    other's potential.  A chain's results do not depend on it. */
  int32_t group;                 /* the group nmx_nuts_step advances (0 .. num_groups - 1) */
  /* Per-leaf decision trace (parity tests and bench parity legs; NULL = off).  For arena
   * chains c < trace_chains and transitions it0 <= t < it0 + trace_iters, leaf n < trace_leaves
   * of the transition (n counted over the whole tree) writes NMX_TRACE_REC floats at
   * trace[((t - it0) * trace_chains + c) * trace_leaves + n][.] (enum nmx_trace_field): the
   * quantities the reference's decisions at that leaf are taken on (hmc_util.py:851-894
   * leaf energy, :749-764 transition probabilities, :735-746 U-turn dots), so a transition
   * whose path leaves the oracle's can be located at its first differing leaf.  Writing
   * does not change any result. */
  int32_t trace_chains;
  int32_t trace_it0;
  int32_t trace_iters;
  int32_t trace_leaves;
  float* trace;
} nmx_nuts_config;

#define NMX_TRACE_REC 8
enum nmx_trace_field {
  NMX_T_DE = 0,      /* leaf delta energy (NaN -> +inf), hmc_util.py:868-871 */
  NMX_T_P_LEAF,      /* uniform (in-subtree) transition probability; -1 for a subtree's first leaf */
  NMX_T_DOT_SUB,     /* min of the iterative U-turn dots checked at this leaf (+inf: none) */
  NMX_T_P_BIASED,    /* at a subtree end: min(1, exp(w_sub - w_tree)) before turning/diverging
                        zero it; -1 elsewhere */
  NMX_T_DOT_TREE,    /* at a subtree end completed by size: min whole-tree U-turn dot; +inf elsewhere */
  NMX_T_FLAGS,       /* bits: nmx_trace_flag */
  NMX_T_PE,          /* potential energy of the leaf */
  NMX_T_LEAF         /* leaf index in the transition (as float) */
};
enum nmx_trace_flag {
  NMX_TF_TAKE_LEAF = 1, NMX_TF_TURN_SUB = 2, NMX_TF_DIVERGE = 4, NMX_TF_DONE_SUB = 8,
  NMX_TF_TAKE_BIASED = 16, NMX_TF_TURN_TREE = 32, NMX_TF_ITER_DONE = 64
};

/* D-slices of the wide step (0 when dim is small enough for the fused one-kernel step).
 * Depends on dim only, so results never depend on how chains are sharded. */
int nmx_nuts_num_slices(int dim);
/* Arena size/offsets for (C, D, max_depth_alloc, iter_capacity). */
size_t nmx_nuts_arena_bytes(int num_chains, int dim, int max_depth_alloc, int iter_capacity);
int nmx_nuts_field_info(int num_chains, int dim, int max_depth_alloc, int iter_capacity,
                        int field, size_t* offset, size_t* nbytes);

/* Reset adaptation + scalar state: warmup_adapter init_fn (hmc_util.py:546-594) with
 * step_size and an optional diag inverse mass matrix [D] (NULL = ones).  Sets every chain
 * to NMX_PH_NEEDINIT, iteration 0. */
int nmx_nuts_reset(const nmx_nuts_config* cfg, void* arena, float step_size,
                   const float* inverse_mass_diag, void* stream);
/* init_to_uniform draw for chains in NEEDINIT (numpyro/infer/initialization.py:95-129,
 * find_valid_initial_params attempt loop infer/util.py:386-388): z_eval ~ U(-radius, radius),
 * phase -> INITEVAL. */
int nmx_nuts_init_draw(const nmx_nuts_config* cfg, void* arena, int attempt, float radius,
                       void* stream);
/* User init params z [D][ldc] for every chain: z_eval = z, phase -> INITEVAL. */
int nmx_nuts_init_from(const nmx_nuts_config* cfg, void* arena, const float* z, void* stream);
/* Validity check after the potential ran (infer/util.py:437-444): finite U and grad ->
 * state (z, grad, U) stored, phase START; otherwise NEEDINIT.  counters[1] = #NEEDINIT. */
int nmx_nuts_init_check(const nmx_nuts_config* cfg, void* arena, void* stream);
/* Set every non-DONE chain with a stored state to START and extend iter_end; used when a
 * run continues from post_warmup_state / last_state (mcmc.py:664-670). */
int nmx_nuts_resume(const nmx_nuts_config* cfg, void* arena, void* stream);
/* find_reasonable_step_size (numpyro/infer/hmc_util.py:314-384), run by warmup_adapter at
 * init (:573-576) and at the end of every middle adaptation window (:619-626) when
 * find_heuristic_step_size (hmc.py:320-331): begin resets every chain's search; each round is
 * propose (step *= 2^direction, momentum r = M^-1 eps as the reference draws it, first half
 * step -> z_eval; searching chains listed in active list 0, count in counters[2]) -> the
 * model's potential on that list -> finish (second half step, dE, new direction; a chain that
 * stops stores its step size and restarts dual averaging there, at_init selecting
 * log(10 step) or log(10) + log(step)).  counters[1] = chains still searching. */
int nmx_heuristic_begin(const nmx_nuts_config* cfg, void* arena, void* stream);
int nmx_heuristic_propose(const nmx_nuts_config* cfg, void* arena, void* stream);
int nmx_heuristic_finish(const nmx_nuts_config* cfg, void* arena, int at_init, void* stream);
/* Dense mass (whitened arena, unit_mass): noise writes each searching chain's normals eps
 * [D][ldc] (the draw propose would make; 0 for the others), the caller maps them to the
 * whitened momentum p = T^T M^-1 eps (z = mu + T w: the reference's r = M^-1 eps,
 * hmc_util.py:359, with kinetic 0.5 r^T M^-1 r = 0.5 |p|^2), and propose_with runs propose
 * with that momentum ([D][ldc]; NULL = propose). */
int nmx_heuristic_noise(const nmx_nuts_config* cfg, void* arena, float* eps, void* stream);
int nmx_heuristic_propose_with(const nmx_nuts_config* cfg, void* arena, const float* momentum, void* stream);
/* One lockstep step of the per-chain NUTS/HMC state machine (sample_kernel hmc.py:459-530
 * with build_tree hmc_util.py:1088-1180 unrolled into leaves): consumes the potential at
 * z_eval for LEAF chains, advances trees / transitions / adaptation / collection, and
 * writes the next z_eval.  samples: [collection_size][D][ldc] (constrained via transform,
 * int8 [D]: 0 identity, 1 exp; NULL: no draws are written, only the fields);
 * fields: [collection_size][NMX_NUM_COLLECT][ldc].
 * dim <= 256: one fused kernel; dim >= 257: three D-split kernels (leapfrog end + partial
 * dots / fixed-order reduction + scalar logic / apply), same results semantics. */
int nmx_nuts_step(const nmx_nuts_config* cfg, void* arena, float* samples, float* fields,
                  const int8_t* transform, void* stream);

/* The step of the wide schedule (dim >= 257) fused with the potential of a D-split model:
 * ONE call replaces `potential(z_eval) -> nmx_nuts_step` of the launched loop (the model's
 * value_and_grad, hmc_util.py:242-252, then the leapfrog end / tree / transition logic of
 * nmx_nuts_step) with three kernels instead of six: the model's row gradients fused with the
 * leapfrog end of the same rows (per D-slice), a fixed-order slice reduction whose last block
 * per chain group finishes U, the scalar-site gradients and the scalar logic, and the apply
 * kernel.  Loop: nmx_nuts_resume, nmx_nuts_step once (starts the transitions), then this call
 * until counters[0] == num_chains.  Same semantics as the launched loop; sums in a fixed
 * order that depends on dim only (rounding differs from the separate kernels).
 *   NMX_WIDE_STOCHASTIC_VOLATILITY: data = returns[n], dim == n + 2 (stochastic_volatility.py:57-65)
 *   NMX_WIDE_FUNNEL:                data unused, n == dim (funnel.py:44-46)
 *   NMX_WIDE_FUNNEL_NONCENTERED:    data unused, n == dim (funnel.py:49, LocScaleReparam(0))
 * workspace: nmx_nuts_wide_model_workspace_bytes(dim, num_chains) bytes, zero-filled before
 * the first call (the library leaves its arrival counters zero). */
#define NMX_WIDE_STOCHASTIC_VOLATILITY 1
#define NMX_WIDE_FUNNEL 2
#define NMX_WIDE_FUNNEL_NONCENTERED 3
size_t nmx_nuts_wide_model_workspace_bytes(int dim, int num_chains);
int nmx_nuts_step_wide_model(const nmx_nuts_config* cfg, void* arena, float* samples, float* fields,
                             const int8_t* transform, int model, const float* data, int n, void* workspace,
                             void* stream);

/* Persistent per-chain schedule for the D-split models: ONE launch
 * runs every remaining transition of [iter_begin, iter_end) of every chain (or max_steps
 * leaves per chain; relaunch until counters[0] == num_chains), one workgroup per chain: the
 * model's row gradients fused with the leapfrog end, a block reduction, the potential's
 * finish and the tree / transition / adaptation logic, then the proposal / momentum / next
 * position rows -- the whole of `potential(z_eval) -> nmx_nuts_step` per leaf without a host
 * loop, D-slices or chain groups (a chain never waits for another).  Models and data as
 * nmx_nuts_step_wide_model.  Needs cfg->layout = NMX_LAYOUT_CHAIN_ROWS (the arena written by
 * nmx_nuts_reset / init_* with that layout) and cfg->sync_chains = 0 (the lockstep schedule
 * is one launch per transition: iter_end = iter_begin + 1).  Sums are in an order fixed by
 * dim, so draws do not depend on the number of chains or devices; they differ from the
 * launched wide schedule in rounding.  samples [collection_size][D][ldc] as nmx_nuts_step. */
int nmx_nuts_run_wide(const nmx_nuts_config* cfg, void* arena, float* samples, float* fields,
                      const int8_t* transform, int model, const float* data, int n, int max_steps, void* stream);

/* Persistent schedule for one-wave models (dim < 16): ONE launch runs
 * every remaining transition of [iter_begin, iter_end) of every chain -- each thread owns a
 * chain and alternates the model's potential (inline) with the fused step until the chain is
 * DONE (or max_steps leapfrog steps), replacing the host loop of nmx_nuts_step / potential
 * launches for tiny models such as README.md's eight schools (numpyro/infer/mcmc.py:461-513
 * _single_chain_mcmc + util.py:277-407 fori_collect over hmc.py:459-530 sample_kernel).  The
 * device code is the launched path's, so draws are bitwise identical to it.  Per-chain async
 * only (cfg->sync_chains = 0); call nmx_nuts_resume first, read counters[0] (DONE) after.
 *   model NMX_SMALL_DIAG_NORMAL:   p0 = mu[n], p1 = prec[n], n = dim
 *   model NMX_SMALL_EIGHT_SCHOOLS: p0 = y[J], p1 = sigma[J], n = J = dim - 2 */
#define NMX_SMALL_DIAG_NORMAL 1
#define NMX_SMALL_EIGHT_SCHOOLS 2
int nmx_nuts_run_small(const nmx_nuts_config* cfg, void* arena, float* samples, float* fields,
                       const int8_t* transform, int model, const float* p0, const float* p1, int n, int max_steps,
                       void* stream);

/* ======================================================================================
 * Fused potential-energy + gradient kernels.  Each replaces, for one model,
 * jax.value_and_grad(potential_fn) (numpyro/infer/hmc_util.py:242-252) over
 * potential_energy (numpyro/infer/util.py:302-327).  They evaluate every chain whose
 * phase >= NMX_PH_LEAF and write pe_eval[c] = U(z_c), g_eval[d][c] = dU/dz_d.
 * ====================================================================================== */
typedef struct nmx_eval_batch {
  const float* z;          /* [D][ldc] positions (arena NMX_F_Z_EVAL) */
  float* grad;             /* [D][ldc] (arena NMX_F_G_EVAL) */
  float* pe;               /* [ldc]    (arena NMX_F_PE_EVAL) */
  const int32_t* phase;    /* [ldc]    (arena NMX_F_PHASE); NULL = evaluate every chain */
  const int32_t* active_idx;   /* optional compacted chain list (arena NMX_F_ACTIVE_IDX);
                                  when set, only chains active_idx[0 .. *active_count) are
                                  evaluated and `phase` is ignored */
  const int32_t* active_count;
  int32_t num_chains;      /* without a list: positions >= num_chains hold no chain; with a
                              list: an upper bound on *active_count that kernels may size their
                              grids by (the engine lowers it as chains finish) */
  int32_t ldc;
} nmx_eval_batch;

/* Unnormalized diagonal Gaussian, U = 0.5 sum((z-mu)^2 * prec): the test target of
 * test/infer/test_mcmc.py:28-72. */
int nmx_pe_diag_normal(const float* mu, const float* prec, int dim, const nmx_eval_batch* ev,
                       void* stream);
/* Eight schools, centred (README.md:47-55), z = (mu, log tau, theta[J]). */
int nmx_pe_eight_schools(const float* y, const float* sigma, int J, const nmx_eval_batch* ev,
                         void* stream);

/* Stochastic volatility (examples/stochastic_volatility.py:57-65): sigma ~ Exponential(50),
 * s ~ GaussianRandomWalk(sigma, T), nu ~ Exponential(0.1), r ~ StudentT(nu, 0, exp(s));
 * z = (log nu, s[T], log sigma).  HBM-bound stencil, lgamma/digamma for nu. */
int nmx_pe_stochastic_volatility(const float* returns, int T, const nmx_eval_batch* ev, void* workspace,
                                 void* stream);
/* Centred funnel (examples/funnel.py:44-46): y ~ N(0,3), x ~ N(0, exp(y/2))^(dim-1);
 * z = (x[dim-1], y). */
int nmx_pe_funnel(int dim, const nmx_eval_batch* ev, void* workspace, void* stream);
/* Non-centred funnel: examples/funnel.py:49 reparam(model, config={"x": LocScaleReparam(0)})
 * (numpyro/infer/reparam.py:104-145, centered = 0): x_decentered ~ N(0,1)^(dim-1), y ~ N(0,3);
 * z = (x_decentered[dim-1], y); the deterministic site x = exp(y/2) x_decentered is formed
 * host side.  Replaces value_and_grad of the reparameterized potential_fn. */
int nmx_pe_funnel_noncentered(int dim, const nmx_eval_batch* ev, void* workspace, void* stream);
/* Workspace (per-slice partial sums) of the three kernels above for num_chains chains. */
size_t nmx_pe_wide_workspace_bytes(int dim, int num_chains);

/* Bayesian neural network (examples/bnn.py:43-74): X [N][Dx], Y [N] (D_Y = 1), H hidden
 * units, tanh; z = (log prec_obs, w1[Dx][H], w2[H][H], w3[H]).  One workgroup per evaluated
 * chain with weights and activations in LDS (needs 4 (Dx H + H^2 + H + N Dx + 2N + 2 N H + 256)
 * bytes <= 160 KiB). */
int nmx_pe_bnn(const float* X, const float* Y, int N, int Dx, int H, const nmx_eval_batch* ev, void* workspace,
               void* stream);
/* nmx_pe_bnn on operands already in rows: position p of the batch reads z_rows[p][0..D) and
 * writes g_rows[p][0..D) (D = 1 + Dx H + H^2 + H; pe to ev->pe[chain(p)]), without the
 * column <-> row transposes (the whitened dense path hands its products over in rows). */
int nmx_pe_bnn_rows(const float* X, const float* Y, int N, int Dx, int H, const nmx_eval_batch* ev,
                    const float* z_rows, float* g_rows, void* stream);
/* Workspace of nmx_pe_bnn: the evaluated chains' z and gradient transposed to rows. */
size_t nmx_pe_bnn_workspace_bytes(int Dx, int H, int num_chains);

/* Logistic regression (examples/covtype.py:66-71): coefs ~ N(0,1)^D,
 * obs ~ BernoulliLogits(X @ coefs).  X is first packed (row tiles with the label in a pad
 * column); U and dU are computed by two f32 MFMA GEMMs per 32-row tile
 * (X.Z and X^T.(sigmoid(X.Z) - y)) with the logits never leaving registers, per-split
 * partial slabs, then a fixed-order reduction. */
size_t nmx_logreg_packed_bytes(int64_t n_rows, int dim);
int nmx_logreg_pack(const float* X, const float* y, int64_t n_rows, int dim, void* packed,
                    void* stream);
size_t nmx_logreg_workspace_bytes(int64_t n_rows, int dim, int num_chains);
int nmx_logreg_pe_grad(const void* packed, int64_t n_rows, int dim, const nmx_eval_batch* ev,
                       void* workspace, void* stream);
/* Number of row splits the kernel uses for n_rows (depends on n_rows only, so results
 * do not depend on how many chains or GPUs share the work). */
int nmx_logreg_num_splits(int64_t n_rows);

/* ---- dense mass matrix (hmc_util.py:1203-1220 dense matvecs, hmc.py:103-108 momentum,
 *      hmc_util.py:612-620 dense Welford finalize) ----
 * With inverse mass M^-1 = T T^T, NUTS with dense mass on z is NUTS with identity mass on
 * w, z = mu + T w (kinetic energy, U-turn dot products and momentum draws map exactly;
 * with T = tril_inv^T the whitened momentum is the reference's `eps`).  Each leapfrog then
 * costs z = mu + T w and g_w = T^T g_z, two chain-batched products:
 *   Out[i][c] = sum_k At[k][i] * In[k][c] (+ bias[i])
 * over every 64-chain tile holding a chain with phase[c] >= NMX_PH_LEAF (phase NULL: all);
 * with active_count set, In/Out are packed columns and tiles c0 < *active_count run.
 * At = A^T row-major with leading dimension lda (multiple of 128, >= padded dim) and zero
 * padding in rows/columns >= dim; In/Out are [dim][ldc] chain-major; f32 MFMA.
 * triangle: 0 dense A; 1 A upper triangular; 2 A lower triangular (all-zero K-tiles are
 * skipped: half the MFMA work for T w and T^T g). */
int nmx_dense_padded_dim(int dim);
int nmx_gemm_chains(const float* At, int lda, int dim, const float* In, float* Out, const float* bias,
                    int triangle, int ldc, const int32_t* phase, const int32_t* active_count, int num_chains,
                    void* workspace, void* stream);
/* Workspace for split-K (K split in a number of parts that depends on dim only; partials
 * summed in a fixed order).  0 = no split; a NULL workspace also disables it. */
size_t nmx_gemm_chains_workspace_bytes(int dim, int ldc);
/* The same products f32-accurate on the bf16 matrix cores (split-bf16: each f32 operand as
 * three bf16 terms, six bf16 products per 16-deep k-step, f32 accumulation; the scheme of the
 * covtype kernel).  A is packed once into MFMA-fragment order (Ap, nmx_gemm_x3_packed_a_bytes
 * = 6 lda^2 bytes; At as for nmx_gemm_chains, re-pack whenever At changes); each call splits
 * In into `split` (nmx_gemm_x3_split_bytes(lda, ldc)) and runs the product with the tiles,
 * triangle skipping, split-K workspace (nmx_gemm_chains_workspace_bytes) and fixed-order
 * reduction of nmx_gemm_chains.  Requires 6 lda^2 and 6 lda ldc < 2^31. */
size_t nmx_gemm_x3_packed_a_bytes(int lda);
int nmx_gemm_x3_pack_a(const float* At, int lda, void* Ap, void* stream);
size_t nmx_gemm_x3_split_bytes(int lda, int ldc);
int nmx_gemm_chains_x3(const void* Ap, int lda, int dim, const float* In, float* Out, const float* bias,
                       int triangle, int ldc, const int32_t* phase, const int32_t* active_count, int num_chains,
                       void* split, void* workspace, void* stream);
/* nmx_gemm_chains_x3 with In gathered from a chain-row arena field: column p of the operand is
 * rows[list[p]][0..dim) (p < *active_count; [ldc][dim] rows, NMX_LAYOUT_CHAIN_ROWS) -- the
 * nmx_pack_rows + nmx_gemm_chains_x3 pair in one call, bitwise the same product columns. */
int nmx_gemm_chains_x3_rows(const void* Ap, int lda, int dim, const float* rows, const int32_t* list, float* Out,
                            const float* bias, int triangle, int ldc, const int32_t* active_count, int num_chains,
                            void* split, void* workspace, void* stream);
/* nmx_gemm_chains_x3 with the product column p (< *active_count) stored to the chain-row arena
 * row rows[list[p]][0..dim) (and pe_out[list[p]] = pe_in[p] when pe_in is given) -- the
 * nmx_gemm_chains_x3 + nmx_unpack_rows pair in one call; never K-split (no workspace), so for
 * dim <= 16384 bitwise the same values. */
int nmx_gemm_chains_x3_to_rows(const void* Ap, int lda, int dim, const float* In, const int32_t* list, float* rows,
                               const float* bias, int triangle, int ldc, const int32_t* active_count, int num_chains,
                               void* split, const float* pe_in, float* pe_out, void* stream);
/* The general form of the two above: In gathered from rows through in_list (or [dim][ldc]
 * columns when NULL), Out stored to rows through out_list (or columns when NULL); positions
 * < *active_count; pe_out[out_list[p]] = pe_in[p] when pe_in is given.  Never K-split. */
int nmx_gemm_chains_x3_lists(const void* Ap, int lda, int dim, const float* In, const int32_t* in_list, float* Out,
                             const int32_t* out_list, const float* bias, int triangle, int ldc,
                             const int32_t* active_count, int num_chains, void* split, const float* pe_in,
                             float* pe_out, void* stream);
/* Column compaction around the dense products: packed[d][p] = in[d][list[p]] and back
 * (p < *count, device-side count, grid sized for ldo / ldi positions). */
int nmx_pack_columns(const float* in, int ldi, int dim, const int32_t* list, const int32_t* count, float* out,
                     int ldo, void* stream);
int nmx_unpack_columns(const float* in, int ldi, int dim, const int32_t* list, const int32_t* count, float* out,
                       int ldo, const float* pe_in, float* pe_out, void* stream);
/* The same compaction for a chain-row arena field in ([ldc][dim] rows, NMX_LAYOUT_CHAIN_ROWS):
 * pack_rows: out[d][p] = in[list[p]][d]; unpack_rows: out[list[p]][d] = in[d][p] (+ pe). */
int nmx_pack_rows(const float* in, int ldc, int dim, const int32_t* list, const int32_t* count, float* out,
                  int ldo, void* stream);
int nmx_unpack_rows(const float* in, int ldi, int dim, const int32_t* list, const int32_t* count, float* out,
                    int ldc, const float* pe_in, float* pe_out, void* stream);
/* Per-chain dense mass matrices (the reference's per-chain adaptation, hmc.py:790-798 vmapped
 * init_kernel; hmc_util.py:133-239 welford_covariance(diagonal=False)); these two: dim <= 256.
 * nmx_chain_matvec: out[a][c] = sum_b M[c][b][a] in[b][c] for the listed chains (list/count),
 * or the chains with phase >= LEAF (list NULL; phase NULL = every chain < num_chains);
 * M [C][dim][dim] f32: T_c^T row-major gives z = T_c w, T_c row-major gives g_w = T_c^T g_z.
 * nmx_chain_welford: welford update_fn (:172-196) of every chain with its draw z [dim][ldc],
 * n = the count after this draw; mean [C][dim], m2 [C][dim][dim] (row a = delta_post[a] *
 * delta_pre). */
int nmx_chain_matvec(const float* M, int dim, const float* in, float* out, int ldc, const int32_t* list,
                     const int32_t* count, const int32_t* phase, int num_chains, void* stream);
int nmx_chain_welford(const float* z, int dim, int ldc, int num_chains, int n, float* mean, float* m2,
                      void* stream);
/* The same for dim <= 4096 (the same hmc.py:790-798 / hmc_util.py:133-239 semantics; above dim
 * 256 a workgroup per (chain, 256 outputs) and a two-launch Welford).  tri: 0 full M, 1 forward
 * with T_c upper triangular (M = T_c^T: rows b < a are zero), 2 backward (M = T_c: rows b > a
 * are zero) -- the zero rows are skipped.  nmx_chain_welford_ws needs `work` of
 * nmx_chain_welford_work_bytes(dim, num_chains) bytes (0 up to dim 256). */
int nmx_chain_matvec_tri(const float* M, int dim, const float* in, float* out, int ldc, const int32_t* list,
                         const int32_t* count, const int32_t* phase, int num_chains, int tri, void* stream);
size_t nmx_chain_welford_work_bytes(int dim, int num_chains);
int nmx_chain_welford_ws(const float* z, int dim, int ldc, int num_chains, int n, float* mean, float* m2,
                         float* work, void* stream);
/* Multivariate normal, U = 0.5 (z-mu)^T P (z-mu), grad = P z - P mu (one nmx_gemm_chains
 * with At = P^T, bias = -P mu) then the per-chain quadratic form: the dense-mass test
 * targets of test/infer/test_mcmc.py:73-100 and :313-343. */
int nmx_pe_mvn(const float* prec_t, int lda, const float* mu, const float* neg_prec_mu, int dim,
               const nmx_eval_batch* ev, void* stream);

/* ---- posterior predictive (numpyro/infer/util.py:888-1090 Predictive, :803-885
 *      _predictive: the model re-run with the latent sites substituted from each posterior
 *      sample, observed sites sampled).  Samples are constrained values, [num_samples][...]
 *      row-major; draws are Philox-keyed by (seed, sample, element). ---- */
/* examples/covtype.py:66-71: obs ~ Bernoulli(logits = X @ coefs); X [n_rows][dim] f32,
 * coefs [num_samples][dim], out [num_samples][n_rows] int32 0/1. */
int nmx_predict_logreg(const float* X, int64_t n_rows, int dim, const float* coefs, int num_samples,
                       uint64_t seed, int32_t* out, void* stream);
/* README.md:47-55 eight schools: obs ~ Normal(loc, scale); loc [num_samples][n] (theta),
 * scale [n] (sigma), out [num_samples][n]. */
int nmx_predict_normal(const float* loc, const float* scale, int n, int num_samples, uint64_t seed,
                       float* out, void* stream);
/* examples/bnn.py:43-74: Y ~ Normal(tanh(tanh(X w1) w2) w3, 1/sqrt(prec_obs)); X [n][dx];
 * samples [num_samples][1 + dx*dh + dh*dh + dh*dy] (prec_obs, w1, w2, w3: sorted sites);
 * out [num_samples][n][dy]. */
int nmx_predict_bnn(const float* X, int n, int dx, int dh, int dy, const float* samples, int num_samples,
                    uint64_t seed, float* out, void* stream);

/* ---- self tests (no reference counterpart; used by tests and smoke()) ---- */
/* Philox4x32-10 on device: ctr_key is n x {c0,c1,c2,c3,k0,k1}, out is n x 4 words. */
int nmx_selftest_philox(const uint32_t* ctr_key, uint32_t* out, int n, void* stream);
/* C[32][32] = A[32][K] * B[K][32] through v_mfma_f32_32x32x2_f32 (fragment-layout probe). */
int nmx_selftest_mfma(const float* A, const float* B, float* C, int K, void* stream);
/* Probe of the debug build's device checks (NMX_DCHECK): value != 0 prints a failed check from
 * the device in libnumpyro_amd_debug.so.  Returns 1 in the debug build, 0 in the release build,
 * a negative status on a launch error. */
int nmx_selftest_dcheck(int value, void* stream);
/* nmx_expf_unchecked (the stochastic-volatility row's exp, nmx_wide_models.h) and the device expf
 * at n points: fast[i], ref[i] (bitwise equal for |x| <= 87). */
int nmx_selftest_expf(const float* x, float* fast, float* ref, int n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NUMPYRO_AMD_H */
