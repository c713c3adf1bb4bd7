// Vectorized-chain NUTS / HMC as a per-chain state machine on the GPU.
//
// The reference builds a NUTS tree with nested lax.while_loops under vmap
// (numpyro/infer/hmc_util.py:984-1180); under vmap every chain runs until the slowest
// chain of the batch is done ("lockstep").  Here a tree is unrolled into
// leaves: one nmx_nuts_step launch consumes one potential evaluation per LEAF chain and
// advances that chain's tree, transition, adaptation and collection, then writes the next
// position to evaluate.  A chain whose transition ends starts its next transition in the
// same launch (sync_chains=0), so the potential kernel always has a full batch; the
// per-chain computation, and with it every output, is identical to the lockstep
// schedule (sync_chains=1) because all randomness is keyed per chain (nmx_common.h).
//
// Layout: chain-major SoA.  Block = 64 chains x TPC waves; wave w handles coordinates
// d = w, w+TPC, ... of its 64 chains and dot products are reduced across the TPC waves
// through LDS in a fixed order (deterministic).
#include <math.h>
#include <string.h>

#include <type_traits>

#include "nmx_api_internal.h"
#include <stdlib.h>

#include "nmx_common.h"
#include "nmx_small_models.h"
#include "nmx_wide_models.h"

namespace {

constexpr int MAXD = NMX_MAX_TREE_DEPTH;
constexpr int NPART = 2 * MAXD + 3;  // KE, checkpoint dots (2 per level), whole-tree dots
constexpr int WIDE_MIN_D = 257;      // D from which the step runs D-split (wide schedule)
#ifndef NMX_STEP_CPW
#define NMX_STEP_CPW 16
#endif
constexpr int STEP_CPW = NMX_STEP_CPW;  // chains per wave of the fused step (TPC = 8, D >= 16)
constexpr int SMALL_CPW = 16;        // chains per wave of the one-wave step (D < 16) and persistent kernel

// slice width of the wide schedule: 32 (D < 4096) and 64 measured best over 16-256
// 64 from D = 2048: SV (D = 2519) at 8192 chains 4.49M vs 4.36M leapfrog/s at 32, at 1024 chains
// 3.89M vs 3.93M (fused wide step); narrower models keep 32 (more blocks per chain group)
inline int slice_width(int D) { return D >= 2048 ? 64 : 32; }
inline int num_slices(int D) { return D >= WIDE_MIN_D ? (D + slice_width(D) - 1) / slice_width(D) : 0; }
constexpr size_t ALIGN = 256;

inline size_t align_up(size_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }
inline int ldc_of(int C) { return (C + 63) / 64 * 64; }

constexpr int NUM_INT_SCALARS = NMX_F_ACT_WFN - NMX_F_PHASE + 1;
constexpr int NUM_FLOAT_SCALARS = NMX_F_PE_EVAL - NMX_F_STEP_SIZE + 1;
constexpr int NUM_VECTORS = NMX_F_G_EVAL - NMX_F_Z + 1;

size_t field_bytes(int field, int ldc, int D, int MD, int iter_cap) {
  if (field <= NMX_F_ACT_WFN) return (size_t)ldc * 4;
  if (field <= NMX_F_PE_EVAL) return (size_t)ldc * 4;
  if (field <= NMX_F_G_EVAL) return (size_t)D * ldc * 4;
  if (field <= NMX_F_CKPT_RSUM) return (size_t)MD * D * ldc * 4;
  if (field == NMX_F_ACTIVE_IDX) return (size_t)2 * ldc * 4;
  if (field == NMX_F_COUNTERS) return 16 * 4;
  if (field == NMX_F_FINISHED) return (size_t)(iter_cap > 0 ? iter_cap : 1) * 4;
  if (field == NMX_F_PART) return (size_t)num_slices(D) * NPART * ldc * 4;
  if (field == NMX_F_PART0) return (size_t)num_slices(D) * ldc * 4;
  if (field == NMX_F_TOT) return num_slices(D) > 0 ? (size_t)(NPART + 1) * ldc * 4 : 0;
  return 0;
}

size_t field_offset(int field, int ldc, int D, int MD, int iter_cap) {
  size_t off = 0;
  for (int f = 0; f < field; ++f) off += align_up(field_bytes(f, ldc, D, MD, iter_cap));
  return off;
}

// Device view of the arena.  The per-chain scalar fields are consecutive arrays of ldc
// entries and the vector fields consecutive arrays of D * ldc (field_offset), so a field is
// its group's base + index * stride: two pointers and two strides instead of a pointer per
// field (a persistent kernel's loop would otherwise hold ~60 loop-invariant pointers).
struct Arena {
  char* sbase;       // field NMX_F_PHASE; scalar field f at sbase + (f - NMX_F_PHASE) * sstride
  char* vbase;       // field NMX_F_Z; vector field f at vbase + (f - NMX_F_Z) * vstride
  size_t sstride, vstride;
  float* ckr;
  float* ckrs;
  int32_t* active_idx;
  int32_t* counters;
  int32_t* finished;
  float* part;
  float* part0;
  float* tot;
};

// Keeps a base pointer in SGPRs across a loop (the empty asm stops the compiler from hoisting the
// field addresses derived from it, which overflowed the SGPRs) without losing its global address
// space: the round trip goes through an address_space(1) value, so accesses through the pointer
// still compile to global loads / stores with an SGPR base and a VGPR offset.  A plain generic
// pointer through the asm became opaque and every arena access a flat one -- two VGPRs of
// address each, and flat loads count against the LDS counter too, so each LDS read waited for
// the HBM loads in flight (the persistent wide kernel: 76 flat loads and 127 flat stores).
template <class T>
__device__ __forceinline__ void pin_sgpr_global(T*& p) {
  auto* g = (__attribute__((address_space(1))) T*)p;
  asm volatile("" : "+s"(g));
  p = (T*)g;
}

#define AI(f) reinterpret_cast<int32_t*>(a.sbase + (size_t)((f) - NMX_F_PHASE) * a.sstride)
#define AF(f) reinterpret_cast<float*>(a.sbase + (size_t)((f) - NMX_F_PHASE) * a.sstride)
#define AV(f) reinterpret_cast<float*>(a.vbase + (size_t)((f) - NMX_F_Z) * a.vstride)

// the strided form above is exact: every scalar field spans ldc * 4 bytes and every vector
// field D * ldc * 4, both multiples of ALIGN (ldc % 64 == 0), laid out in enum order
static_assert(NMX_F_PHASE == 0 && NMX_F_STEP_SIZE == NMX_F_ACT_WFN + 1 && NMX_F_Z == NMX_F_PE_EVAL + 1,
              "scalar fields must precede the vector fields contiguously");

Arena make_arena(void* base, int ldc, int D, int MD, int iter_cap) {
  Arena a;
  char* b = (char*)base;
  a.sbase = b + field_offset(NMX_F_PHASE, ldc, D, MD, iter_cap);
  a.vbase = b + field_offset(NMX_F_Z, ldc, D, MD, iter_cap);
  a.sstride = (size_t)ldc * 4;
  a.vstride = (size_t)D * ldc * 4;
  a.ckr = (float*)(b + field_offset(NMX_F_CKPT_R, ldc, D, MD, iter_cap));
  a.ckrs = (float*)(b + field_offset(NMX_F_CKPT_RSUM, ldc, D, MD, iter_cap));
  a.active_idx = (int32_t*)(b + field_offset(NMX_F_ACTIVE_IDX, ldc, D, MD, iter_cap));
  a.counters = (int32_t*)(b + field_offset(NMX_F_COUNTERS, ldc, D, MD, iter_cap));
  a.finished = (int32_t*)(b + field_offset(NMX_F_FINISHED, ldc, D, MD, iter_cap));
  a.part = (float*)(b + field_offset(NMX_F_PART, ldc, D, MD, iter_cap));
  a.part0 = (float*)(b + field_offset(NMX_F_PART0, ldc, D, MD, iter_cap));
  a.tot = (float*)(b + field_offset(NMX_F_TOT, ldc, D, MD, iter_cap));
  return a;
}

// chain groups of the launched fused step (nmx_nuts_config.num_groups)
__host__ __device__ __forceinline__ int group_count(const nmx_nuts_config& cfg) {
  return cfg.num_groups > 1 ? cfg.num_groups : 1;
}
__host__ __device__ __forceinline__ int group_size(const nmx_nuts_config& cfg) {
  const int g = group_count(cfg);
  return (cfg.num_chains + g - 1) / g;
}
__host__ __device__ __forceinline__ int group_first(const nmx_nuts_config& cfg) {
  return group_count(cfg) > 1 ? cfg.group * group_size(cfg) : 0;
}
// index of the group's list-length counter of a parity
__host__ __device__ __forceinline__ int list_counter(const nmx_nuts_config& cfg, int parity) {
  return 2 + 2 * (group_count(cfg) > 1 ? cfg.group : 0) + parity;
}

struct StepArgs {
  Arena a;
  nmx_nuts_config cfg;
  float* samples;
  float* fields;
  const int8_t* transform;
};

// Fixed-order sum of N partials over the NV "virtual waves" of a block that hold the same
// chain (virtual wave vw = wave * SUBS + sub, chain slot cl = lane % CPW; all get the total).
// Must be reached by every thread of the block.
// workgroup barrier ordering LDS accesses only (global memory operations may stay in flight)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// LDS floats vblock_sum<NV, CPW, N> uses: every caller sizes its array with this (the NV >= 8
// form also keeps the N x CPW totals behind the partials)
template <int NV, int CPW, int N>
constexpr int vblock_lds_floats() {
  return NV >= 8 ? N * NV * CPW + N * CPW : (NV > 1 ? N * NV * CPW : 1);
}
// floats of the fused step's reduction array (its largest vblock_sum: N = NPART)
template <int TPC, int CPW>
constexpr int step_lds_floats() {
  return vblock_lds_floats<TPC * (64 / CPW), CPW, NPART>();
}

template <int NV, int CPW, int N>
__device__ __forceinline__ void vblock_sum(float (&v)[N], float* lds, int vw, int cl) {
  if constexpr (NV >= 8) {
    // the block's NV x CPW threads share the N x CPW sums (each over the NV partials in slice
    // order, as below), then every thread reads its chain's totals: NV + N LDS reads per thread
    // instead of N x NV (the fused covtype step, NV = 32, N = 23: 55 instead of 736, which made
    // the reduction ~25k cycles of a ~30k-cycle tail-launch block -- s_memtime stamps).  Same
    // order, bitwise the same sums.  lds holds N x NV x CPW partials + N x CPW totals.
    // LDS-only barriers: __syncthreads' workgroup fence would first wait for every global store
    // the leaf / apply rows issued (vmcnt(0): a store round trip per barrier); no thread of the
    // launched step reads global data another thread wrote in the same launch (a chain's lanes
    // own their rows in both row phases: leaf_rows / apply_rows give row d of chain c to one
    // lane in both, and that rule must hold for any change there), so only the LDS partials
    // need ordering
    constexpr int NT = NV * CPW;
#pragma unroll
    for (int i = 0; i < N; ++i) lds[(i * NV + vw) * CPW + cl] = v[i];
    lds_barrier();
    float* const tot = lds + N * NV * CPW;
    for (int o = threadIdx.x; o < N * CPW; o += NT) {
      const int i = o / CPW, c = o % CPW;
      float s = 0.0f;
#pragma unroll 8
      for (int w = 0; w < NV; ++w) s += lds[(i * NV + w) * CPW + c];
      tot[o] = s;
    }
    lds_barrier();
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = tot[i * CPW + cl];
    // the next call writes the partials only, and reads them after its first barrier
  } else if constexpr (NV > 1) {
#pragma unroll
    for (int i = 0; i < N; ++i) lds[(i * NV + vw) * CPW + cl] = v[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < N; ++i) {
      float s = 0.0f;
#pragma unroll 4
      for (int w = 0; w < NV; ++w) s += lds[(i * NV + w) * CPW + cl];
      v[i] = s;
    }
    __syncthreads();
  }
}

// Fixed-order sum of N per-thread partials over the TPC waves of a block (all waves get
// the total).  Must be reached by every thread of the block.
template <int TPC, int N>
__device__ __forceinline__ void block_sum(float (&v)[N], float* lds) {
  if constexpr (TPC > 1) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < N; ++i) lds[(i * TPC + wv) * 64 + lane] = v[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < N; ++i) {
      float s = 0.0f;
#pragma unroll
      for (int w = 0; w < TPC; ++w) s += lds[(i * TPC + w) * 64 + lane];
      v[i] = s;
    }
    __syncthreads();
  }
}

__device__ __forceinline__ float transform_value(int8_t code, float z) {
  return code == 1 ? expf(z) : z;
}

// ---------------------------------------------------------------------------------------
// The step.
//
// Per-chain scalar state is loaded into registers before the first barrier, updated
// identically by all waves of a block (decisions only depend on block-reduced sums and
// the chain's own registers) and written back by wave 0 only, so no wave can observe
// another wave's partial update.  Vector work is split by coordinate.
//
// The scalar logic (leaf_phase / tree_phase) is shared by two schedules of the same step:
//  * fused: one kernel, block = 64 chains x TPC waves owning all D coordinates (small D);
//  * wide (D >= WIDE_MIN_D): V1 (leapfrog end + partial dots per D-slice) -> S (fixed-order
//    reduction + scalar logic, one block per 64 chains) -> V2 (apply the decisions per
//    D-slice), so the grid is chain-groups x D-slices and fills the GPU at any C.
// ---------------------------------------------------------------------------------------
struct ChainScalars {
  int phase, it, depth, sub_n, dir, tree_n, widx, da_t, wf_n, turning, tree_div, sub_div;
  int hmc_k, hmc_n, last_nsteps, last_div, maxdepth;
  float step, E0, pe, energy, tree_w, tree_acc, sub_w, sub_acc, pe_sub, e_sub;
  float da_xt, da_xavg, da_gavg, da_prox, mean_acc, last_acc, step_eff;
};

__device__ __forceinline__ void load_scalars(const Arena& a, int c, ChainScalars& s) {
  s.phase = AI(NMX_F_PHASE)[c];
  s.it = AI(NMX_F_ITER)[c];
  s.depth = AI(NMX_F_DEPTH)[c];
  s.sub_n = AI(NMX_F_SUB_N)[c];
  s.dir = AI(NMX_F_DIR)[c];
  s.tree_n = AI(NMX_F_TREE_N)[c];
  s.widx = AI(NMX_F_WINDOW_IDX)[c];
  s.da_t = AI(NMX_F_DA_T)[c];
  s.wf_n = AI(NMX_F_WF_N)[c];
  s.turning = AI(NMX_F_TURNING)[c];
  s.tree_div = AI(NMX_F_TREE_DIV)[c];
  s.sub_div = AI(NMX_F_SUB_DIV)[c];
  s.hmc_k = AI(NMX_F_HMC_K)[c];
  s.hmc_n = AI(NMX_F_HMC_N)[c];
  s.last_nsteps = AI(NMX_F_LAST_NSTEPS)[c];
  s.last_div = AI(NMX_F_LAST_DIV)[c];
  s.maxdepth = AI(NMX_F_MAXDEPTH_CUR)[c];
  s.step = AF(NMX_F_STEP_SIZE)[c];
  s.E0 = AF(NMX_F_E0)[c];
  s.pe = AF(NMX_F_PE)[c];
  s.energy = AF(NMX_F_ENERGY)[c];
  s.tree_w = AF(NMX_F_TREE_W)[c];
  s.tree_acc = AF(NMX_F_TREE_ACC)[c];
  s.sub_w = AF(NMX_F_SUB_W)[c];
  s.sub_acc = AF(NMX_F_SUB_ACC)[c];
  s.pe_sub = AF(NMX_F_PE_SUB)[c];
  s.e_sub = AF(NMX_F_E_SUB)[c];
  s.da_xt = AF(NMX_F_DA_XT)[c];
  s.da_xavg = AF(NMX_F_DA_XAVG)[c];
  s.da_gavg = AF(NMX_F_DA_GAVG)[c];
  s.da_prox = AF(NMX_F_DA_PROX)[c];
  s.mean_acc = AF(NMX_F_MEAN_ACC)[c];
  s.last_acc = AF(NMX_F_LAST_ACC)[c];
  s.step_eff = AF(NMX_F_STEP_EFF)[c];
}

__device__ __forceinline__ void store_scalars(const Arena& a, int c, const ChainScalars& s) {
  AI(NMX_F_PHASE)[c] = s.phase;
  AI(NMX_F_ITER)[c] = s.it;
  AI(NMX_F_DEPTH)[c] = s.depth;
  AI(NMX_F_SUB_N)[c] = s.sub_n;
  AI(NMX_F_DIR)[c] = s.dir;
  AI(NMX_F_TREE_N)[c] = s.tree_n;
  AI(NMX_F_WINDOW_IDX)[c] = s.widx;
  AI(NMX_F_DA_T)[c] = s.da_t;
  AI(NMX_F_WF_N)[c] = s.wf_n;
  AI(NMX_F_TURNING)[c] = s.turning;
  AI(NMX_F_TREE_DIV)[c] = s.tree_div;
  AI(NMX_F_SUB_DIV)[c] = s.sub_div;
  AI(NMX_F_HMC_K)[c] = s.hmc_k;
  AI(NMX_F_HMC_N)[c] = s.hmc_n;
  AI(NMX_F_LAST_NSTEPS)[c] = s.last_nsteps;
  AI(NMX_F_LAST_DIV)[c] = s.last_div;
  AI(NMX_F_MAXDEPTH_CUR)[c] = s.maxdepth;
  AF(NMX_F_STEP_SIZE)[c] = s.step;
  AF(NMX_F_E0)[c] = s.E0;
  AF(NMX_F_PE)[c] = s.pe;
  AF(NMX_F_ENERGY)[c] = s.energy;
  AF(NMX_F_TREE_W)[c] = s.tree_w;
  AF(NMX_F_TREE_ACC)[c] = s.tree_acc;
  AF(NMX_F_SUB_W)[c] = s.sub_w;
  AF(NMX_F_SUB_ACC)[c] = s.sub_acc;
  AF(NMX_F_PE_SUB)[c] = s.pe_sub;
  AF(NMX_F_E_SUB)[c] = s.e_sub;
  AF(NMX_F_DA_XT)[c] = s.da_xt;
  AF(NMX_F_DA_XAVG)[c] = s.da_xavg;
  AF(NMX_F_DA_GAVG)[c] = s.da_gavg;
  AF(NMX_F_DA_PROX)[c] = s.da_prox;
  AF(NMX_F_MEAN_ACC)[c] = s.mean_acc;
  AF(NMX_F_LAST_ACC)[c] = s.last_acc;
  AF(NMX_F_STEP_EFF)[c] = s.step_eff;
}

// Decisions of one step for one chain.
struct Act {
  bool leaf, take_leaf, done_sub, take_biased, hmc_accept, iter_done, wf_update, finalize;
  bool tree_chk;  // this leaf completes its subtree by size: the whole-tree U-turn dots are needed
  bool start_iter, prep_leaf, fin_done, fin_wait, div_new;
  int dirR, new_dir, k, j, imin, imax, slot, fin_t, wfn;
  float pe_eval, E_new, acc_new, w_new, p_leaf;
};

enum : int {
  ACT_TAKE_LEAF = 1 << 0, ACT_DONE_SUB = 1 << 1, ACT_TAKE_BIASED = 1 << 2, ACT_HMC_ACCEPT = 1 << 3,
  ACT_ITER_DONE = 1 << 4, ACT_WF_UPDATE = 1 << 5, ACT_FINALIZE = 1 << 6, ACT_START = 1 << 7,
  ACT_PREP = 1 << 8, ACT_DIRR = 1 << 9, ACT_NEWDIR = 1 << 10, ACT_KE0_PENDING = 1 << 11,
};

__device__ __forceinline__ int pack_act(const Act& A) {
  return (A.take_leaf ? ACT_TAKE_LEAF : 0) | (A.done_sub ? ACT_DONE_SUB : 0) |
         (A.take_biased ? ACT_TAKE_BIASED : 0) | (A.hmc_accept ? ACT_HMC_ACCEPT : 0) |
         (A.iter_done ? ACT_ITER_DONE : 0) | (A.wf_update ? ACT_WF_UPDATE : 0) |
         (A.finalize ? ACT_FINALIZE : 0) | (A.start_iter ? ACT_START : 0) | (A.prep_leaf ? ACT_PREP : 0) |
         (A.dirR ? ACT_DIRR : 0) | (A.new_dir ? ACT_NEWDIR : 0) | (A.start_iter ? ACT_KE0_PENDING : 0);
}

// The step's decisions known before the leaf: from the chain's phase ph and its scalars.
__device__ __forceinline__ void begin_act(const nmx_nuts_config& cfg, const ChainScalars& S, int ph, Act& A) {
  A = Act{};
  A.leaf = ph == NMX_PH_LEAF;
  A.start_iter = ph == NMX_PH_START;
  A.dirR = A.leaf ? S.dir : 0;
  A.new_dir = A.dirR;
  A.slot = -1;
  A.imin = 1;
  A.imax = 0;
  const bool is_nuts = cfg.algo == NMX_ALGO_NUTS;
  A.k = (A.leaf && is_nuts) ? S.sub_n : 0;
  A.j = (A.leaf && is_nuts) ? S.depth : 0;
  if (A.leaf && is_nuts) nmx_leaf_idx_to_ckpt_idxs(A.k, A.imin, A.imax);  // :1036
  A.tree_chk = A.leaf && is_nuts && (A.k + 1 == (1 << A.j));
  // the checkpoint rows a leaf touches exist: imax <= depth < max_depth_alloc
  NMX_DCHECK(!(A.leaf && is_nuts) || (A.imax < cfg.max_depth_alloc && A.j < cfg.max_depth_alloc));
}

// Whether a chain waiting at the end of its transition (sync_chains) may start the next one:
// every chain of the job has finished that transition.  The count is written by other blocks
// (and, with chain groups, other streams) while this launch runs, so two loads of it can
// disagree: a chain whose threads span several waves must take this decision ONCE and share
// it (fused_step: through LDS, k_chain_step: one thread), or some of its waves start the
// transition (momentum, first half step) while others keep waiting -- the round-5 lockstep
// chain-group failure, one 16-chain block of k_nuts_step<8,16> drawing differently.
__device__ __forceinline__ bool wait_released(const nmx_nuts_config& cfg, const Arena& a, int it) {
  const int slot_w = it - 1 - cfg.iter_begin;
  const int fin = (slot_w >= 0 && slot_w < cfg.iter_capacity)
                      ? __hip_atomic_load(&a.finished[slot_w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : cfg.num_chains;
  return fin >= cfg.num_chains;
}

// Resolve WAIT (sync_chains) and set up the step's inputs.  resolve_wait = false leaves a
// waiting chain in WAIT (begin_act: no work); the caller then decides for the chain as a whole
// (wait_released above).  Only schedules with one lane per chain, or all of a chain's lanes in
// one wave (one load instruction serves them all), resolve here.
__device__ __forceinline__ int begin_step(const nmx_nuts_config& cfg, const Arena& a, int c, bool valid,
                                          ChainScalars& S, Act& A, bool resolve_wait = true) {
  // the leaf's potential is loaded with the scalars, whatever the phase (a load behind the
  // phase test would be one more dependent memory round per step)
  float pe_ev = 0.0f;
  if (valid) {
    load_scalars(a, c, S);
    pe_ev = AF(NMX_F_PE_EVAL)[c];
  } else {
    S.phase = NMX_PH_DONE;
  }
  int ph = S.phase;
  if (ph == NMX_PH_WAIT && resolve_wait && wait_released(cfg, a, S.it)) ph = NMX_PH_START;
  begin_act(cfg, S, ph, A);
  A.pe_eval = A.leaf ? pe_ev : 0.0f;
  return ph;
}

// Leaf scalars (_build_basetree, hmc_util.py:851-894) and the NUTS leaf bookkeeping of
// _iterative_build_subtree (:999-1061) that only needs the kinetic energy.
__device__ __forceinline__ void leaf_phase(const nmx_nuts_config& cfg, ChainScalars& S, Act& A, float ke,
                                           uint64_t seed, uint32_t gch) {
  if (!A.leaf) return;
  A.E_new = A.pe_eval + ke;
  float dE = A.E_new - S.E0;
  if (isnan(dE)) dE = INFINITY;
  A.w_new = -dE;
  A.div_new = dE > cfg.max_delta_energy;
  A.acc_new = fminf(expf(-dE), 1.0f);
  if (cfg.algo != NMX_ALGO_NUTS) return;
  const int k = A.k, j = A.j;
  if (k == 0) {  // new_tree = new_leaf (:1019-1021)
    A.take_leaf = true;
    A.p_leaf = -1.0f;
    S.sub_w = A.w_new;
    S.sub_acc = A.acc_new;
  } else {  // _combine_tree(..., biased_transition=False) (:767-848, :749-753)
    const float p = nmx_sigmoid(A.w_new - S.sub_w);
    const float u = nmx_u01(nmx_rng(seed, gch, S.it, NMX_EV_LEAF, j, k).x);
    A.take_leaf = u < p;
    A.p_leaf = p;
    S.sub_w = nmx_logaddexp(S.sub_w, A.w_new);
    S.sub_acc = S.sub_acc + A.acc_new;
  }
  S.sub_div = A.div_new;
  S.sub_n = k + 1;
  if (A.take_leaf) {
    S.pe_sub = A.pe_eval;
    S.e_sub = A.E_new;
  }
}

// Everything after the U-turn dots: subtree end / tree combine, HMC accept, transition end
// (adaptation scalars, mean accept prob, collection slot + fields), next transition or
// doubling.  turn(i, side) = reduced checkpoint dot, tree(side) = reduced tree dot.
template <class TurnF, class TreeF>
__device__ __forceinline__ void tree_phase(const nmx_nuts_config& cfg, ChainScalars& S, Act& A, TurnF turn,
                                           TreeF tree, uint64_t seed, uint32_t gch, float* fields, int c,
                                           bool writer) {
  const bool is_nuts = cfg.algo == NMX_ALGO_NUTS;
  const int ldc = cfg.ldc;
  float it_accept = 0.f;
  int it_nsteps = 0;
  bool it_div = false;
  bool new_doubling = false;
  if (A.leaf && is_nuts) {
    const int leaf_n = S.tree_n + A.k;  // leaf index in the transition (trace)
    const int leaf_it = S.it;
    float pb_raw = -1.0f;
    bool turning_sub = false;
#pragma unroll
    for (int i = 0; i < MAXD; ++i)
      if (i >= A.imin && i <= A.imax) turning_sub |= (turn(i, 0) <= 0.0f) | (turn(i, 1) <= 0.0f);
    A.done_sub = (S.sub_n >= (1 << A.j)) || turning_sub || A.div_new;  // loop exit (:992-997)
    if (A.done_sub) {
      // _double_tree -> _combine_tree(..., biased_transition=True) (:936-938, :756-764)
      // the whole-tree check is only decisive when the subtree completed by size; a subtree
      // stopped by a U-turn or a divergence ends the transition either way (tree.turning is
      // internal state, not an output)
      const bool turning_tree = turning_sub || (A.tree_chk && ((tree(0) <= 0.0f) || (tree(1) <= 0.0f)));
      float pb = expf(S.sub_w - S.tree_w);
      pb = isnan(pb) ? pb : fminf(pb, 1.0f);  // jnp.clip keeps NaN
      pb_raw = pb;
      if (turning_sub || A.div_new) pb = 0.0f;
      const float u = nmx_u01(nmx_rng(seed, gch, S.it, NMX_EV_BIASED, A.j, 0).x);
      A.take_biased = u < pb;
      if (A.take_biased) {
        S.pe = S.pe_sub;
        S.energy = S.e_sub;
      }
      S.depth = A.j + 1;
      S.tree_w = nmx_logaddexp(S.tree_w, S.sub_w);
      S.tree_div = A.div_new;
      S.tree_acc = S.tree_acc + S.sub_acc;
      S.tree_n = S.tree_n + S.sub_n;
      S.turning = turning_tree;
      // build_tree loop condition (:1153-1157)
      if (S.depth >= S.maxdepth || turning_tree || A.div_new) {
        A.iter_done = true;
        it_accept = S.tree_acc / (float)S.tree_n;  // _nuts_next :441
        it_nsteps = S.tree_n;
        it_div = A.div_new;
      } else {
        new_doubling = true;
      }
    } else {
      A.prep_leaf = true;
    }
    // decision trace (cfg.trace, parity tests): the quantities of this leaf's decisions
    if (cfg.trace != nullptr && writer && c < cfg.trace_chains && leaf_it >= cfg.trace_it0 &&
        leaf_it < cfg.trace_it0 + cfg.trace_iters && leaf_n < cfg.trace_leaves) {
      float dmin_sub = INFINITY, dmin_tree = INFINITY;
#pragma unroll
      for (int i = 0; i < MAXD; ++i)
        if (i >= A.imin && i <= A.imax) dmin_sub = fminf(dmin_sub, fminf(turn(i, 0), turn(i, 1)));
      if (A.done_sub && A.tree_chk && !turning_sub && !A.div_new) dmin_tree = fminf(tree(0), tree(1));
      const int fl = (A.take_leaf ? NMX_TF_TAKE_LEAF : 0) | (turning_sub ? NMX_TF_TURN_SUB : 0) |
                     (A.div_new ? NMX_TF_DIVERGE : 0) | (A.done_sub ? NMX_TF_DONE_SUB : 0) |
                     (A.take_biased ? NMX_TF_TAKE_BIASED : 0) | (S.turning && A.done_sub ? NMX_TF_TURN_TREE : 0) |
                     (A.iter_done ? NMX_TF_ITER_DONE : 0);
      float* R = cfg.trace + (((size_t)(leaf_it - cfg.trace_it0) * cfg.trace_chains + c) * cfg.trace_leaves + leaf_n) *
                                 NMX_TRACE_REC;
      R[NMX_T_DE] = -A.w_new;
      R[NMX_T_P_LEAF] = A.p_leaf;
      R[NMX_T_DOT_SUB] = dmin_sub;
      R[NMX_T_P_BIASED] = pb_raw;
      R[NMX_T_DOT_TREE] = dmin_tree;
      R[NMX_T_FLAGS] = (float)fl;
      R[NMX_T_PE] = A.pe_eval;
      R[NMX_T_LEAF] = (float)leaf_n;
    }
  }
  // HMC leaf bookkeeping (_hmc_next, hmc.py:364-414)
  if (A.leaf && !is_nuts) {
    S.hmc_k = S.hmc_k + 1;
    if (S.hmc_k < S.hmc_n) {
      A.prep_leaf = true;
    } else {
      const float u = nmx_u01(nmx_rng(seed, gch, S.it, NMX_EV_ACCEPT, 0, 0).x);
      A.hmc_accept = u < A.acc_new;
      // decision trace: one record per HMC transition (leaf 0), the end point's delta energy
      // and the Metropolis accept probability it is decided on
      if (cfg.trace != nullptr && writer && c < cfg.trace_chains && S.it >= cfg.trace_it0 &&
          S.it < cfg.trace_it0 + cfg.trace_iters && cfg.trace_leaves > 0) {
        float* R = cfg.trace + ((size_t)(S.it - cfg.trace_it0) * cfg.trace_chains + c) * cfg.trace_leaves *
                                   NMX_TRACE_REC;
        R[NMX_T_DE] = -A.w_new;
        R[NMX_T_P_LEAF] = A.acc_new;
        R[NMX_T_DOT_SUB] = INFINITY;
        R[NMX_T_P_BIASED] = -1.0f;
        R[NMX_T_DOT_TREE] = INFINITY;
        R[NMX_T_FLAGS] = (float)((A.hmc_accept ? NMX_TF_TAKE_LEAF : 0) | (A.div_new ? NMX_TF_DIVERGE : 0) |
                                 NMX_TF_DONE_SUB | NMX_TF_ITER_DONE);
        R[NMX_T_PE] = A.pe_eval;
        R[NMX_T_LEAF] = 0.0f;
      }
      if (A.hmc_accept) {
        S.pe = A.pe_eval;
        S.energy = A.E_new;
      } else {
        S.energy = S.E0;
      }
      A.iter_done = true;
      it_accept = A.acc_new;
      it_nsteps = S.hmc_n;
      it_div = A.div_new;
    }
  }
  // transition end: warmup_adapter update_fn (hmc_util.py:637-705), mean accept prob
  // (hmc.py:509-513), collection slot.
  if (A.iter_done) {
    const int t = S.it;
    A.fin_t = t;
    if (t < cfg.num_warmup) {
      float new_step = S.step;
      if (cfg.adapt_step_size) {  // dual_averaging update_fn (:103-126)
        S.da_t = S.da_t + 1;
        const float g = cfg.target_accept_prob - it_accept;
        const float tt0 = (float)(S.da_t + 10);
        S.da_gavg = (1.0f - 1.0f / tt0) * S.da_gavg + g / tt0;
        S.da_xt = S.da_prox - sqrtf((float)S.da_t) / 0.05f * S.da_gavg;
        const float weight_t = powf((float)S.da_t, -0.75f);
        S.da_xavg = (1.0f - weight_t) * S.da_xavg + weight_t * S.da_xt;
        new_step = (t == cfg.num_warmup - 1) ? expf(S.da_xavg) : expf(S.da_xt);  // :662-666
        new_step = fminf(fmaxf(new_step, 1.17549435e-38f), 3.40282347e+38f);  // :670-672
      }
      const int widx = S.widx;
      const bool middle = (0 < widx) && (widx < cfg.num_windows - 1);
      A.wf_update = cfg.adapt_mass_matrix && middle;
      if (A.wf_update) S.wf_n = S.wf_n + 1;
      const bool at_end = t == cfg.window_end[widx];
      S.widx = widx + (at_end ? 1 : 0);
      A.finalize = at_end && middle && cfg.adapt_mass_matrix;  // _update_at_window_end (:596-635)
      if (at_end && middle && cfg.adapt_step_size) {
        S.da_prox = logf(10.0f) + logf(new_step);
        S.da_xt = 0.0f;
        S.da_xavg = 0.0f;
        S.da_gavg = 0.0f;
        S.da_t = 0;
      }
      S.step = new_step;
    }
    A.wfn = S.wf_n;
    if (A.finalize) S.wf_n = 0;
    const int itr = t + 1;
    const int nn = t < cfg.num_warmup ? itr : itr - cfg.num_warmup;
    S.mean_acc = S.mean_acc + (it_accept - S.mean_acc) / (float)nn;
    S.last_acc = it_accept;
    S.last_nsteps = it_nsteps;
    S.last_div = it_div;
    S.it = itr;
    // fori_collect slot (numpyro/util.py:330-346): idx = (i - start) // thinning, last write wins
    if (cfg.collection_size > 0 && t >= cfg.collect_start) {
      const int off = t - cfg.collect_start;
      if (off % cfg.collect_thinning == cfg.collect_thinning - 1) {
        const int s = off / cfg.collect_thinning;
        if (s < cfg.collection_size) A.slot = s;
      }
    }
    NMX_DCHECK(A.slot < cfg.collection_size);
    if (A.slot >= 0 && writer) {
      float* F = fields + (size_t)A.slot * NMX_NUM_COLLECT * ldc;
      F[NMX_C_POTENTIAL_ENERGY * ldc + c] = S.pe;
      F[NMX_C_ENERGY * ldc + c] = S.energy;
      F[NMX_C_ACCEPT_PROB * ldc + c] = it_accept;
      F[NMX_C_MEAN_ACCEPT_PROB * ldc + c] = S.mean_acc;
      F[NMX_C_STEP_SIZE * ldc + c] = S.step;
      F[NMX_C_NUM_STEPS * ldc + c] = (float)it_nsteps;
      F[NMX_C_DIVERGING * ldc + c] = it_div ? 1.0f : 0.0f;
      F[NMX_C_ITER * ldc + c] = (float)itr;
    }
    if (itr >= cfg.iter_end) {
      S.phase = NMX_PH_DONE;
      A.fin_done = true;
    } else if (cfg.sync_chains) {
      S.phase = NMX_PH_WAIT;
      A.fin_wait = true;
    } else {
      A.start_iter = true;
    }
  }
  // new transition: tree init (sample_kernel hmc.py:471-481, build_tree :1127-1151), first
  // direction; new doubling direction (:1160-1162).
  if (A.start_iter) {
    if (is_nuts) {
      S.step_eff = S.step;
      S.maxdepth = S.it < cfg.num_warmup ? cfg.max_tree_depth_warmup : cfg.max_tree_depth;  // hmc.py:488-490
      A.new_dir = nmx_u01(nmx_rng(seed, gch, S.it, NMX_EV_DIRECTION, 0, 0).x) < 0.5f;
    } else {
      int n;
      if (cfg.num_steps > 0) n = cfg.num_steps;
      else n = (int)ceilf(cfg.trajectory_length / S.step);  // _get_num_steps hmc.py:85-89
      n = n < 1 ? 1 : n;
      S.step_eff = cfg.trajectory_length > 0.0f ? cfg.trajectory_length / (float)n : S.step;
      S.hmc_n = n;
      S.hmc_k = 0;
      A.new_dir = 1;
    }
    S.depth = 0;
    S.sub_n = 0;
    S.tree_n = 0;
    S.turning = 0;
    S.tree_div = 0;
    S.tree_w = 0.0f;
    S.tree_acc = 0.0f;
    S.dir = A.new_dir;
    S.phase = NMX_PH_LEAF;
  } else if (new_doubling) {
    A.new_dir = nmx_u01(nmx_rng(seed, gch, S.it, NMX_EV_DIRECTION, S.depth, 0).x) < 0.5f;
    S.dir = A.new_dir;
    S.sub_n = 0;
    A.prep_leaf = true;
  }
  if (A.prep_leaf) S.phase = NMX_PH_LEAF;
}

// End of step, wave 0: write scalars back, DONE / sync counters, compacted list.
__device__ __forceinline__ void end_step(const nmx_nuts_config& cfg, const Arena& a, int c, bool valid, int ph_in,
                                         const ChainScalars& S, const Act& A, bool list = true) {
  if (valid) {
    if (S.phase != ph_in || A.leaf || A.start_iter || A.iter_done) store_scalars(a, c, S);
    if (A.fin_done) {
      atomicAdd(&a.counters[0], 1);
      if (group_count(cfg) > 1) atomicAdd(&a.counters[10 + cfg.group], 1);  // the group's own count
    }
    if (A.fin_wait) {
      const int fs = A.fin_t - cfg.iter_begin;
      if (fs >= 0 && fs < cfg.iter_capacity) atomicAdd(&a.finished[fs], 1);
    }
  }
  // compacted list of chains whose next leaf is pending: the potential kernels then cost
  // in proportion to the chains still integrating.  List order is arbitrary; a chain's
  // result does not depend on its position.
  if (!list) return;  // persistent kernel: the potential runs inline, no list
  const int lane = threadIdx.x & 63;
  const bool pend = valid && (A.start_iter || A.prep_leaf);
  const uint64_t m = __ballot(pend);
  if (m) {
    int base = 0;
    if (lane == __builtin_ctzll(m))
      base = atomicAdd(&a.counters[list_counter(cfg, cfg.parity)], __builtin_popcountll(m));
    base = __shfl(base, __builtin_ctzll(m));
    if (pend) {
      const int pos = base + __builtin_popcountll(m & ((1ull << lane) - 1ull));
      NMX_DCHECK(pos < group_size(cfg));
      a.active_idx[(size_t)cfg.parity * cfg.ldc + group_first(cfg) + pos] = c;
    }
  }
}

// ---- per-coordinate vector bodies shared by both schedules -----------------------------
struct VecCtx {
  const Arena* a;
  int ldc, D;
  size_t ck_stride;
  bool unit;  // cfg.unit_mass: inv_mass == mass_sqrt == 1, not loaded
};

// The frontier (the moving end's position z_eval, its gradient g_eval and its momentum, RR or RL
// by the tree direction) and the inverse mass of the persistent wide kernel's chain, LDS-resident
// when the kernel carries them (k_wide_persistent<..., CARRY>): [D] floats each, row d at byte
// d * 4.  The arena's inverse mass stays authoritative (the window finalize writes both).
struct Front {
  float* z;
  float* g;
  float* r;
  float* im;
};

// L1 + L2 minus the proposal copy: finish the pending leapfrog (hmc_util.py:306-308),
// kinetic energy, subtree r_sum, checkpoints and the U-turn partial dots.
// red[0] = KE partial, red[1 + 2i + side] = checkpoint i, red[1 + 2 MAXD + side] = tree.
// Split into a load stage and a compute/store stage so that several rows' loads are in
// flight before the (possibly aliasing, from the compiler's view) stores.
struct LeafIn {
  float g, rf, im, rs_old, rst, ro;
  float ckr[MAXD], ckrs[MAXD];
};

template <bool NUTS, bool PRE, bool LOADG = true>
__device__ __forceinline__ void leaf_load(const VecCtx& v, const Act& A, uint32_t off, LeafIn& x) {
  const Arena& a = *v.a;
  if constexpr (LOADG) x.g = nmx_at(AV(NMX_F_G_EVAL), off);
  x.rf = nmx_at((A.dirR ? AV(NMX_F_RR) : AV(NMX_F_RL)), off);
  x.im = v.unit ? 1.0f : nmx_at(AV(NMX_F_INV_MASS), off);
  if constexpr (NUTS) {
    x.rs_old = A.k == 0 ? 0.0f : nmx_at(AV(NMX_F_RSUM_SUB), off);
    if (A.tree_chk) {
      x.rst = nmx_at(AV(NMX_F_RSUM), off);
      x.ro = nmx_at((A.dirR ? AV(NMX_F_RL) : AV(NMX_F_RR)), off);  // the other end's momentum
    }
    // checkpoints read by the U-turn check; the range is empty for even leaves, whose
    // checkpoint write below therefore never feeds this step's check (:1036-1047)
#pragma unroll
    for (int i = 0; i < MAXD; ++i) {
      if (PRE && i >= A.imin && i <= A.imax) {
        x.ckr[i] = nmx_at(a.ckr + i * v.ck_stride, off);
        x.ckrs[i] = nmx_at(a.ckrs + i * v.ck_stride, off);
      }
    }
  }
}

template <bool NUTS, bool PRE>
__device__ __forceinline__ void leaf_store(const VecCtx& v, const Act& A, float seff, uint32_t off, const LeafIn& x,
                                           float* red, bool st = true) {
  // st = false: the sums only (the persistent wide kernel's scalar-site rows: every thread
  // adds them to its totals, one thread stores)
  const Arena& a = *v.a;
  const float es = A.dirR ? seff : -seff;
  const float half = 0.5f * es;
  const float r = x.rf - half * x.g;
  if (st) nmx_at((A.dirR ? AV(NMX_F_RR) : AV(NMX_F_RL)), off) = r;
  // the moving end's z / grad stay in Z_EVAL / G_EVAL (the frontier); apply_store saves
  // them into the side arrays only when the next doubling turns around
  const float im = x.im;
  red[0] += (im * r) * r;
  if constexpr (NUTS) {
    const float rs = (A.k == 0) ? r : x.rs_old + r;
    if (st) nmx_at(AV(NMX_F_RSUM_SUB), off) = rs;
    if (st && (A.k & 1) == 0) {  // checkpoint update (:1040-1047)
      nmx_at(a.ckr + A.imax * v.ck_stride, off) = r;
      nmx_at(a.ckrs + A.imax * v.ck_stride, off) = rs;
    }
    // _is_iterative_turning (:961-981): all checkpoints in [imin, imax]; the reference
    // stops at the first turning one, the OR over them is the same predicate.
#pragma unroll
    for (int i = 0; i < MAXD; ++i) {
      if (i >= A.imin && i <= A.imax) {
        const float rl = PRE ? x.ckr[i] : nmx_at(a.ckr + i * v.ck_stride, off);
        const float rsub = (rs - (PRE ? x.ckrs[i] : nmx_at(a.ckrs + i * v.ck_stride, off))) + rl;
        const float rss = rsub - (rl + r) / 2.0f;  // _momentum_angle :735
        red[1 + 2 * i] += (im * rl) * rss;
        red[2 + 2 * i] += (im * r) * rss;
      }
    }
    // whole-tree turning check with the tree's outer momenta (:795-799), at subtree completion
    if (A.tree_chk) {
      const float rst = x.rst + rs;
      const float rlv = A.dirR ? x.ro : r;
      const float rrv = A.dirR ? r : x.ro;
      const float rss2 = rst - (rlv + rrv) / 2.0f;
      red[1 + 2 * MAXD] += (im * rlv) * rss2;
      red[2 + 2 * MAXD] += (im * rrv) * rss2;
    }
  }
}

// rows d0, d0 + step, ... < d1 of chain column c, ROWS rows per iteration.  Row ownership rule
// (the fused step's LDS-only barriers depend on it, vblock_sum): the lane that runs row d of
// chain c here is the one that runs it in apply_rows (same d0 / step), so no lane ever reads a
// global value another lane of the launch wrote.
template <bool NUTS, int ROWS, bool PRE1 = (ROWS == 2)>
__device__ __forceinline__ void leaf_rows(const VecCtx& v, const Act& A, float seff, int d0, int d1, int step, int c,
                                          float* red) {
  int d = d0;
  if constexpr (ROWS == 3) {
    // software-pipelined: the next row's loads are issued before this row's stores, so two
    // rows' loads are in flight through the whole loop (one row per round leaves the memory
    // pipe idle while a row computes and stores)
    if (d >= d1) return;
    LeafIn cur;
    uint32_t ic = nmx_row_off(d, v.ldc, c);
    leaf_load<NUTS, true>(v, A, ic, cur);
    for (; d < d1; d += step) {
      const int dn = d + step;
      const uint32_t in = nmx_row_off(dn, v.ldc, c);
      LeafIn nxt;
      if (dn < d1) leaf_load<NUTS, true>(v, A, in, nxt);
      leaf_store<NUTS, true>(v, A, seff, ic, cur, red);
      cur = nxt;
      ic = in;
    }
    return;
  }
  if constexpr (ROWS == 2) {
    for (; d + step < d1; d += 2 * step) {
      LeafIn x0, x1;
      const uint32_t i0 = nmx_row_off(d, v.ldc, c), i1 = nmx_row_off(d + step, v.ldc, c);
      leaf_load<NUTS, true>(v, A, i0, x0);
      leaf_load<NUTS, true>(v, A, i1, x1);
      leaf_store<NUTS, true>(v, A, seff, i0, x0, red);
      leaf_store<NUTS, true>(v, A, seff, i1, x1, red);
    }
  }
  for (; d < d1; d += step) {
    LeafIn x0;
    const uint32_t i0 = nmx_row_off(d, v.ldc, c);
    leaf_load<NUTS, PRE1>(v, A, i0, x0);
    leaf_store<NUTS, PRE1>(v, A, seff, i0, x0, red);
  }
}

// Proposal copies, tree r_sum, HMC accept copy, Welford / window finalize, collection
// (L3/L4), then the momentum draw + tree init or the next half step and z_eval (L5/L6,
// velocity_verlet first half, hmc_util.py:297-301).  Load stage first (values the
// stores below would otherwise serialise behind), then compute/store.
// Frontier layout: Z_EVAL / G_EVAL hold the moving end of the trajectory (the leaf just
// evaluated); the side arrays Z{L,R} / G{L,R} hold only the end the tree is NOT growing
// from.  R{L,R} hold both ends' momenta.  A turn-around (new doubling direction differs from
// the last leaf's) parks the frontier in its side arrays and loads the other end.
struct ApplyIn {
  float ze, ge;     // frontier = the leaf just evaluated (take_leaf, hmc_accept, prep_leaf)
  float rst, rss;   // tree / subtree r_sum (done_sub)
  float zs, gs;     // subtree proposal (take_biased)
  float zp, gp;     // state
  float wm, w2;     // Welford
  float ms, im;     // mass
  float zfn, rfn, gfn;  // the end the next leaf grows from (prep_leaf)
};

__device__ __forceinline__ bool turn_around(const Act& A) { return A.prep_leaf && A.new_dir != A.dirR; }

// CARRY (the persistent wide kernel with an LDS frontier, row d): the frontier's position,
// gradient and momentum come from and go to fr; the arena's copies are written only where the
// trajectory leaves them behind (a turn-around parks the frontier in its side arrays, RR / RL
// included) and at the kernel's exit
template <bool CARRY = false>
__device__ __forceinline__ void apply_load(const VecCtx& v, const Act& A, uint32_t off, ApplyIn& x,
                                           const Front& fr = {}, int d = 0) {
  const Arena& a = *v.a;
  if (A.take_leaf || A.hmc_accept || A.prep_leaf) {
    if constexpr (CARRY) {
      x.ze = fr.z[d];
      x.ge = fr.g[d];
    } else {
      x.ze = nmx_at(AV(NMX_F_Z_EVAL), off);
      x.ge = nmx_at(AV(NMX_F_G_EVAL), off);
    }
  }
  if (A.done_sub) {
    x.rst = nmx_at(AV(NMX_F_RSUM), off);
    x.rss = nmx_at(AV(NMX_F_RSUM_SUB), off);
  }
  if (A.take_biased && !A.take_leaf) {
    x.zs = nmx_at(AV(NMX_F_ZSUB), off);
    x.gs = nmx_at(AV(NMX_F_GSUB), off);
  }
  const bool need_state = (A.iter_done || A.start_iter) && !A.take_biased && !A.hmc_accept;
  if (need_state) {
    x.zp = nmx_at(AV(NMX_F_Z), off);
    x.gp = nmx_at(AV(NMX_F_ZGRAD), off);
  }
  if (A.wf_update || A.finalize) {
    x.wm = nmx_at(AV(NMX_F_WF_MEAN), off);
    x.w2 = nmx_at(AV(NMX_F_WF_M2), off);
  }
  if (A.start_iter) x.ms = v.unit ? 1.0f : nmx_at(AV(NMX_F_MASS_SQRT), off);
  if (A.start_iter || A.prep_leaf) x.im = v.unit ? 1.0f : (CARRY ? fr.im[d] : nmx_at(AV(NMX_F_INV_MASS), off));
  if (A.prep_leaf) {
    const int nd = A.new_dir;
    if constexpr (CARRY) {
      // the frontier keeps growing: its momentum from LDS, read unconditionally (written as one
      // conditional LDS-or-arena load, the two became a flat load through a selected address)
      x.rfn = fr.r[d];
      if (turn_around(A)) x.rfn = nmx_at((nd ? AV(NMX_F_RR) : AV(NMX_F_RL)), off);
    } else {
      x.rfn = nmx_at((nd ? AV(NMX_F_RR) : AV(NMX_F_RL)), off);
    }
    if (turn_around(A)) {
      x.zfn = nmx_at((nd ? AV(NMX_F_ZR) : AV(NMX_F_ZL)), off);
      x.gfn = nmx_at((nd ? AV(NMX_F_GR) : AV(NMX_F_GL)), off);
    } else {
      x.zfn = x.ze;
      x.gfn = x.ge;
    }
  }
}

// Returns the momentum KE partial (start_iter).
// soff: offset of the row in the samples buffer ([S][D][ldc]; default: off, the arena's layout)
template <bool CARRY = false>
__device__ __forceinline__ float apply_store(const VecCtx& v, const Act& A, float step_eff, int d, uint32_t off,
                                             ApplyIn& x, float mom, float* samp, const int8_t* transform,
                                             const nmx_nuts_config& cfg, uint32_t soff = 0xFFFFFFFFu,
                                             const Front& fr = {}) {
  const Arena& a = *v.a;
  if (A.take_leaf) {
    nmx_at(AV(NMX_F_ZSUB), off) = x.ze;
    nmx_at(AV(NMX_F_GSUB), off) = x.ge;
    x.zs = x.ze;
    x.gs = x.ge;
  }
  if (A.done_sub) nmx_at(AV(NMX_F_RSUM), off) = x.rst + x.rss;
  if (A.take_biased) {
    nmx_at(AV(NMX_F_Z), off) = x.zs;
    nmx_at(AV(NMX_F_ZGRAD), off) = x.gs;
    x.zp = x.zs;
    x.gp = x.gs;
  }
  if (A.hmc_accept) {
    nmx_at(AV(NMX_F_Z), off) = x.ze;
    nmx_at(AV(NMX_F_ZGRAD), off) = x.ge;
    x.zp = x.ze;
    x.gp = x.ge;
  }
  float im = x.im;
  if (A.iter_done) {
    const float z = x.zp;
    if (A.wf_update) {  // welford_covariance update_fn, diagonal (:172-196)
      const float mean = x.wm;
      const float delta_pre = z - mean;
      const float mean_new = mean + delta_pre / (float)A.wfn;
      const float delta_post = z - mean_new;
      x.wm = mean_new;
      x.w2 = x.w2 + delta_pre * delta_post;
      nmx_at(AV(NMX_F_WF_MEAN), off) = x.wm;
      nmx_at(AV(NMX_F_WF_M2), off) = x.w2;
    }
    if (A.finalize) {  // final_fn (:198-237)
      float cov = x.w2 / (float)(A.wfn - 1);
      if (cfg.regularize_mass_matrix) {
        const float scaled = ((float)A.wfn / (float)(A.wfn + 5)) * cov;
        const float shrink = 1e-3f * (5.0f / (float)(A.wfn + 5));
        cov = scaled + shrink;
      }
      im = cov;
      x.ms = 1.0f / sqrtf(cov);
      nmx_at(AV(NMX_F_INV_MASS), off) = cov;
      if constexpr (CARRY) fr.im[d] = cov;
      nmx_at(AV(NMX_F_MASS_SQRT), off) = x.ms;
      nmx_at(AV(NMX_F_WF_MEAN), off) = 0.0f;
      nmx_at(AV(NMX_F_WF_M2), off) = 0.0f;
    }
    if (samp) nmx_at(samp, soff == 0xFFFFFFFFu ? off : soff) = transform_value(transform[d], z);
  }
  float ke0 = 0.0f;
  if (A.start_iter || A.prep_leaf) {
    const int nd = A.new_dir;
    const float es = nd ? step_eff : -step_eff;
    const float half = 0.5f * es;
    float* const ZE = AV(NMX_F_Z_EVAL);
    if (A.start_iter) {
      const float r = x.ms * mom;  // momentum_generator hmc.py:92-110
      const float z = x.zp;
      const float g = x.gp;
      ke0 = (im * r) * r;
      nmx_at(AV(NMX_F_RSUM), off) = r;
      // both ends start at z; only the fixed end goes to the side arrays
      nmx_at((nd ? AV(NMX_F_ZL) : AV(NMX_F_ZR)), off) = z;
      nmx_at((nd ? AV(NMX_F_GL) : AV(NMX_F_GR)), off) = g;
      nmx_at((nd ? AV(NMX_F_RL) : AV(NMX_F_RR)), off) = r;
      const float rh = r - half * g;
      if constexpr (CARRY) {
        fr.r[d] = rh;
        fr.z[d] = z + es * (im * rh);
      } else {
        nmx_at((nd ? AV(NMX_F_RR) : AV(NMX_F_RL)), off) = rh;
        nmx_at(ZE, off) = z + es * (im * rh);
      }
    } else {
      if (turn_around(A)) {
        nmx_at((A.dirR ? AV(NMX_F_ZR) : AV(NMX_F_ZL)), off) = x.ze;
        nmx_at((A.dirR ? AV(NMX_F_GR) : AV(NMX_F_GL)), off) = x.ge;
        if constexpr (CARRY) nmx_at((A.dirR ? AV(NMX_F_RR) : AV(NMX_F_RL)), off) = fr.r[d];
      }
      const float rh = x.rfn - half * x.gfn;
      if constexpr (CARRY) {
        fr.r[d] = rh;
        fr.z[d] = x.zfn + es * (im * rh);
      } else {
        nmx_at((nd ? AV(NMX_F_RR) : AV(NMX_F_RL)), off) = rh;
        nmx_at(ZE, off) = x.zfn + es * (im * rh);
      }
    }
  }
  return ke0;
}

// One block of 4 coordinates (the momentum block), BATCH rows at a time: their loads, then their
// stores (wide schedule: 2; the fused kernel, register-bound: 1).  The momentum KE adds the rows
// in order whatever BATCH is.
template <int BATCH>
__device__ __forceinline__ float apply_block(const VecCtx& v, const Act& A, float step_eff, int blk, int c,
                                             const float (&n)[4], float* samp, const int8_t* transform,
                                             const nmx_nuts_config& cfg) {
  float ke0 = 0.0f;
#pragma unroll
  for (int q0 = 0; q0 < 4; q0 += BATCH) {
    ApplyIn x[BATCH];
#pragma unroll
    for (int q = q0; q < q0 + BATCH; ++q) {
      const int d = 4 * blk + q;
      if (d < v.D) apply_load(v, A, nmx_row_off(d, v.ldc, c), x[q - q0]);
    }
#pragma unroll
    for (int q = q0; q < q0 + BATCH; ++q) {
      const int d = 4 * blk + q;
      if (d < v.D)
        ke0 += apply_store(v, A, step_eff, d, nmx_row_off(d, v.ldc, c), x[q - q0], n[q], samp, transform, cfg);
    }
  }
  return ke0;
}

// Momentum normals of coordinates 4 blk .. 4 blk + 3 (one Philox call per block of 4).
// The key words pass through an empty asm so the Philox key schedule (ten rounds of two keys) is
// computed at the draw: hoisted out of the persistent wide kernel's leaf loop, the 20 round keys
// held SGPRs for the whole launch and pushed its spills into VGPR lanes.  Same values as nmx_rng.
__device__ __forceinline__ void momentum_block(uint64_t seed, uint32_t gch, int it, int blk, float (&n)[4]) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  asm volatile("" : "+s"(k0), "+s"(k1));
  nmx_u4 c;
  c.x = gch;
  c.y = (uint32_t)it;
  c.z = ((uint32_t)NMX_EV_MOMENTUM << 24) | ((uint32_t)blk & 0x00FFFFFFu);
  c.w = 0;
  const nmx_u4 x = nmx_philox4x32_10(c, k0, k1);
  nmx_box_muller(x.x, x.y, n[0], n[1]);
  nmx_box_muller(x.z, x.w, n[2], n[3]);
}

// Rows d0, d0 + step, ... of chain column c, BATCH rows per round: their loads, then the momentum
// normals (the row's Philox block, recomputed per row: ALU that hides the loads' latency), then
// their stores.  The fused kernel's form (TPC > 1): a chain's rows spread evenly over its lanes,
// instead of momentum blocks of four (14 of 32 lanes busy at D = 55, four rounds each).
template <int BATCH>
__device__ __forceinline__ float apply_rows(const VecCtx& v, const Act& A, float step_eff, int d0, int step, int c,
                                            uint64_t seed, uint32_t gch, int it, float* samp,
                                            const int8_t* transform, const nmx_nuts_config& cfg) {
  float ke0 = 0.0f;
  for (int d = d0; d < v.D; d += BATCH * step) {
    ApplyIn x[BATCH];
#pragma unroll
    for (int q = 0; q < BATCH; ++q) {
      const int dq = d + q * step;
      if (dq < v.D) apply_load(v, A, nmx_row_off(dq, v.ldc, c), x[q]);
    }
    float n[BATCH];
#pragma unroll
    for (int q = 0; q < BATCH; ++q) {
      const int dq = d + q * step;
      n[q] = 0.0f;
      if (A.start_iter && dq < v.D) {
        float nb[4];
        momentum_block(seed, gch, it, dq >> 2, nb);
        const int j = dq & 3;
        n[q] = j == 0 ? nb[0] : (j == 1 ? nb[1] : (j == 2 ? nb[2] : nb[3]));
      }
    }
#pragma unroll
    for (int q = 0; q < BATCH; ++q) {
      const int dq = d + q * step;
      if (dq < v.D)
        ke0 += apply_store(v, A, step_eff, dq, nmx_row_off(dq, v.ldc, c), x[q], n[q], samp, transform, cfg);
    }
  }
  return ke0;
}

// ---- fused schedule ----------------------------------------------------------------------
// One fused step for the chains of this block (LIST: append the chains whose next leaf is
// pending to the compacted list; the persistent kernel evaluates inline instead).  A block
// holds CPW chains; each of its TPC waves splits into SUBS = 64 / CPW sub-waves, so a chain's
// coordinates spread over NV = TPC * SUBS lanes: fewer rows per lane (the vector phases are a
// chain of dependent load -> store rounds per row) and C / CPW blocks to spread them over.
// Every lane of a chain runs the chain's scalar logic; one lane (vw == 0) writes it back.
// PA: StepArgs by value for the launched kernel (the kernel argument itself: a reference to it
// made the compiler copy all of it to scratch), a reference to an LDS copy in the persistent
// loop (by value there, the loop-invariant arguments were hoisted into registers and spilled).
template <int TPC, int CPW, bool LIST, class PA>
__device__ __forceinline__ void fused_step(PA P, float* lds, int* wait_go = nullptr) {
  constexpr int SUBS = 64 / CPW;
  constexpr int NV = TPC * SUBS;
  const nmx_nuts_config& cfg = P.cfg;
  const Arena& a = P.a;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int cl = lane % CPW;
  const int vw = wv * SUBS + lane / CPW;
  const int c = group_first(cfg) + blockIdx.x * CPW + cl;
  const int ldc = cfg.ldc;
  const int D = cfg.dim;
  const bool valid = c < cfg.num_chains && c < group_first(cfg) + group_size(cfg);
  const bool is_nuts = cfg.algo == NMX_ALGO_NUTS;
  const uint32_t gch = (uint32_t)(cfg.chain_offset + c);
  const uint64_t seed = cfg.seed;
  // active list [parity ^ 1] was consumed by the previous potential launch; clear it for
  // the next step (which appends to it).  List [parity] was cleared by the previous step.
  if (LIST && blockIdx.x == 0 && threadIdx.x == 0) a.counters[list_counter(cfg, cfg.parity ^ 1)] = 0;

  ChainScalars S;
  Act A;
  // TPC > 1: a chain's lanes span TPC waves; a waiting chain's release is read once, by its
  // virtual wave 0, and published through LDS (read after vblock_sum's barriers; a waiting
  // chain has no leaf, so the rows phase does not depend on it)
  begin_step(cfg, a, c, valid, S, A, TPC == 1);
  if constexpr (TPC > 1) {
    if (vw == 0 && valid && S.phase == NMX_PH_WAIT) wait_go[cl] = wait_released(cfg, a, S.it) ? 1 : 0;
  }
  const int ph_in = S.phase;  // the stored phase (begin_step's return resolves WAIT)
  const VecCtx v{&a, ldc, D, (size_t)D * ldc, cfg.unit_mass != 0};
  const float seff = valid ? S.step_eff : 0.0f;

  float red[NPART];
#pragma unroll
  for (int i = 0; i < NPART; ++i) red[i] = 0.0f;
// two rows per load round in the leaf and apply phases (a lane holds <= 2 rows at D <= 64):
// every row's loads go out before the first row's stores, whose completion the next row's
// loads would otherwise wait for (vmcnt counts stores and loads in issue order); step kernel
// p50 21.0 -> 19.9 us in the 512-chain covtype protocol, bitwise the same draws (round 5)
#ifndef NMX_STEP_LROWS
#define NMX_STEP_LROWS 2
#endif
#ifndef NMX_STEP_AROWS
#define NMX_STEP_AROWS 2
#endif
  constexpr int LROWS = TPC > 1 ? (NMX_STEP_LROWS == 2 ? 2 : 1) : 1;
  constexpr bool LPRE = TPC > 1 && NMX_STEP_LROWS >= 1;
  if (A.leaf) {
    if (is_nuts) leaf_rows<true, LROWS, LPRE>(v, A, seff, vw, D, NV, c, red);
    else leaf_rows<false, LROWS, LPRE>(v, A, seff, vw, D, NV, c, red);
  }
  vblock_sum<NV, CPW, NPART>(red, lds, vw, cl);
  if constexpr (TPC > 1) {
    if (valid && S.phase == NMX_PH_WAIT && wait_go[cl]) begin_act(cfg, S, NMX_PH_START, A);
  }
  leaf_phase(cfg, S, A, 0.5f * red[0], seed, gch);
  tree_phase(
      cfg, S, A, [&](int i, int side) { return red[1 + 2 * i + side]; },
      [&](int side) { return red[1 + 2 * MAXD + side]; }, seed, gch, P.fields, c, vw == 0);

  float ke0[1] = {0.0f};
  const bool vec2 = A.take_leaf || A.done_sub || A.take_biased || A.hmc_accept || A.iter_done || A.start_iter ||
                    A.prep_leaf;
  if (vec2) {
    float* const samp = (A.slot >= 0 && P.samples) ? P.samples + (size_t)A.slot * D * ldc : nullptr;
    const float step_eff = S.step_eff;
    if constexpr (TPC > 1 && NMX_STEP_AROWS >= 1) {
      ke0[0] = apply_rows<NMX_STEP_AROWS>(v, A, step_eff, vw, NV, c, seed, gch, S.it, samp, P.transform, cfg);
    } else {
      for (int blk = vw; 4 * blk < D; blk += NV) {
        float n[4] = {0.f, 0.f, 0.f, 0.f};
        if (A.start_iter) momentum_block(seed, gch, S.it, blk, n);
        ke0[0] += apply_block<1>(v, A, step_eff, blk, c, n, samp, P.transform, cfg);
      }
    }
  }
  vblock_sum<NV, CPW, 1>(ke0, lds, vw, cl);
  if (A.start_iter) {
    S.E0 = S.pe + 0.5f * ke0[0];  // build_tree :1130
    S.energy = S.E0;              // proposal energy of the initial tree (:1137)
  }
  if (vw == 0) end_step(cfg, a, c, valid, ph_in, S, A, LIST);
}

template <int TPC, int CPW>
__global__ __launch_bounds__(64 * TPC) void k_nuts_step(StepArgs P) {
  __shared__ float lds[step_lds_floats<TPC, CPW>()];
  __shared__ int wait_go[CPW];  // sync_chains: the release of each waiting chain (fused_step)
  fused_step<TPC, CPW, true, const StepArgs>(P, lds, wait_go);
}

// ---- persistent schedule for tiny models ----------------------------
// One launch runs every transition of the run: each thread owns a chain and alternates the
// model's potential (inline, per chain) with fused_step<1> until the chain is DONE, so there
// is no host loop, no compacted list and no launch per leapfrog.  The step and the potential
// are the device code of the launched path (k_nuts_step<1>, potential_small.hip), so the
// draws are bitwise those of the launched schedule.  Async schedule only (no sync_chains).
template <class Pot>
__global__ __launch_bounds__(64) void k_nuts_persistent(StepArgs P, Pot pot, int max_steps) {
  __shared__ float lds[step_lds_floats<1, SMALL_CPW>()];
  __shared__ StepArgs sP;
  if (threadIdx.x == 0) sP = P;
  __syncthreads();
  const int c = blockIdx.x * SMALL_CPW + (threadIdx.x & 63) % SMALL_CPW;
  const bool evaluator = (threadIdx.x & 63) < SMALL_CPW;  // one lane per chain runs the potential
  const bool valid = c < P.cfg.num_chains;
  const Arena& a = P.a;
  const int* const phase = AI(NMX_F_PHASE);
  nmx_eval_batch ev;
  ev.z = AV(NMX_F_Z_EVAL);
  ev.grad = AV(NMX_F_G_EVAL);
  ev.pe = AF(NMX_F_PE_EVAL);
  ev.phase = nullptr;
  ev.active_idx = nullptr;
  ev.active_count = nullptr;
  ev.num_chains = P.cfg.num_chains;
  ev.ldc = P.cfg.ldc;
  for (int it = 0; it < max_steps; ++it) {
    const int ph = valid ? phase[c] : NMX_PH_DONE;
    if (!__any(ph != NMX_PH_DONE)) break;  // every chain of the wave finished
    if (ph == NMX_PH_LEAF && evaluator) pot(ev, c);
    __syncthreads();  // the evaluator lane's writes are visible to its chain's other lanes
    fused_step<1, SMALL_CPW, false, const StepArgs&>(sP, lds);
  }
}

// ---- wide schedule -----------------------------------------------------------------------
constexpr int WIDE_WAVES = 4;   // waves per V1/V2 block (64 chains x one D-slice)
constexpr int WIDE_SWAVES = 4;  // waves per S block (slices split across waves)


struct WideArgs {
  StepArgs p;
  int ns;  // slices
  int sw;  // slice width (multiple of 4)
};

__device__ __forceinline__ float* part_ptr(const Arena& a, int ldc, int s, int i) {
  return a.part + ((size_t)s * NPART + i) * ldc;
}

__global__ __launch_bounds__(64 * WIDE_WAVES) void k_wide_v1(WideArgs W) {
  __shared__ float lds[NPART * WIDE_WAVES * 64];
  const nmx_nuts_config& cfg = W.p.cfg;
  const Arena& a = W.p.a;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int s = blockIdx.y;
  const int ldc = cfg.ldc, D = cfg.dim;
  const bool valid = c < cfg.num_chains;
  // every per-chain scalar in one round of loads, ahead of the early exit (a block has only
  // a few rows per wave: a second dependent round was a large share of its time)
  int ph = NMX_PH_DONE, dir = 0, subn = 0, depth = 0;
  float seff0 = 0.0f;
  if (valid) {
    ph = AI(NMX_F_PHASE)[c];
    dir = AI(NMX_F_DIR)[c];
    subn = AI(NMX_F_SUB_N)[c];
    depth = AI(NMX_F_DEPTH)[c];
    seff0 = AF(NMX_F_STEP_EFF)[c];
  }
  if (!__syncthreads_or(ph == NMX_PH_LEAF)) return;
  const bool is_nuts = cfg.algo == NMX_ALGO_NUTS;
  Act A{};
  A.leaf = ph == NMX_PH_LEAF;
  A.dirR = A.leaf ? dir : 0;
  A.k = (A.leaf && is_nuts) ? subn : 0;
  A.j = (A.leaf && is_nuts) ? depth : 0;
  A.imin = 1;
  A.imax = 0;
  if (A.leaf && is_nuts) nmx_leaf_idx_to_ckpt_idxs(A.k, A.imin, A.imax);
  A.tree_chk = A.leaf && is_nuts && (A.k + 1 == (1 << A.j));
  const float seff = A.leaf ? seff0 : 0.0f;
  const VecCtx v{&a, ldc, D, (size_t)D * ldc, cfg.unit_mass != 0};
  float red[NPART];
#pragma unroll
  for (int i = 0; i < NPART; ++i) red[i] = 0.0f;
  const int d0 = s * W.sw, d1 = min(D, d0 + W.sw);
  if (A.leaf) {
    // one row per round with the row's checkpoints loaded ahead: 114 VGPRs, 4 waves per SIMD
    // (rows in pairs: 134 VGPRs, 3 waves; SV launched -2.4%, funnel-10k diag -3.5%)
#ifndef NMX_PX_B
#define NMX_PX_B 2  // rows per thread in flight in the persistent wide kernel (profiles/r03/ab_persistent_occ.txt)
#endif
#ifndef NMX_PX_FAST_APPLY
#define NMX_PX_FAST_APPLY 1  // the persistent wide kernel's mid-trajectory apply loop (persist_apply_prep_rows)
#endif
#ifndef NMX_PX_BA
// rows per thread in flight in the persistent wide kernel's apply phase: SV 8192 chains 1 / 2 / 3 /
// 4 rows 42.7 / 41.9 / 39.7 / 33.9M (profiles/r06/sv_phase_stamps.txt: fewer values live across the
// phase's LDS round trips)
#define NMX_PX_BA 1
#endif
#ifndef NMX_PX_BL
#define NMX_PX_BL NMX_PX_B  // the same in its leaf phase
#endif
#ifndef NMX_V1_ROWS
#define NMX_V1_ROWS 1
#endif
    if (is_nuts) leaf_rows<true, NMX_V1_ROWS, true>(v, A, seff, d0 + wv, d1, WIDE_WAVES, c, red);
    else leaf_rows<false, NMX_V1_ROWS, true>(v, A, seff, d0 + wv, d1, WIDE_WAVES, c, red);
  }
  block_sum<WIDE_WAVES, NPART>(red, lds);
  if (wv == 0 && A.leaf) {
    *(part_ptr(a, ldc, s, 0) + c) = red[0];
    if (is_nuts) {
#pragma unroll
      for (int i = 0; i < MAXD; ++i)
        if (i >= A.imin && i <= A.imax) {
          *(part_ptr(a, ldc, s, 1 + 2 * i) + c) = red[1 + 2 * i];
          *(part_ptr(a, ldc, s, 2 + 2 * i) + c) = red[2 + 2 * i];
        }
      if (A.tree_chk) {
        *(part_ptr(a, ldc, s, 1 + 2 * MAXD) + c) = red[1 + 2 * MAXD];
        *(part_ptr(a, ldc, s, 2 + 2 * MAXD) + c) = red[2 + 2 * MAXD];
      }
    }
  }
}

// Which slice-partial entries chain c needs this step (0: KE, 1..2MAXD: checkpoint pairs,
// 2MAXD+1..+2: tree pair, NPART: momentum KE of a just-started transition).
__device__ __forceinline__ bool entry_needed(const nmx_nuts_config& cfg, const Arena& a, int c, int e) {
  const int ph = AI(NMX_F_PHASE)[c];
  if (e == NPART) return (AI(NMX_F_ACTION)[c] & ACT_KE0_PENDING) != 0;
  if (ph != NMX_PH_LEAF) return false;
  if (e == 0) return true;
  if (cfg.algo != NMX_ALGO_NUTS) return false;
  if (e >= 1 + 2 * MAXD) return AI(NMX_F_SUB_N)[c] + 1 == (1 << AI(NMX_F_DEPTH)[c]);  // tree_chk
  int imin, imax;
  nmx_leaf_idx_to_ckpt_idxs(AI(NMX_F_SUB_N)[c], imin, imax);
  const int i = (e - 1) >> 1;
  return i >= imin && i <= imax;
}

// Fixed-order slice reduction, one block per (64 chains, entry): wave w sums slices w,
// w+4, ... in order, then the waves are added in order.
__global__ __launch_bounds__(64 * WIDE_SWAVES) void k_wide_r(WideArgs W) {
  __shared__ float lds[WIDE_SWAVES * 64];
  const nmx_nuts_config& cfg = W.p.cfg;
  const Arena& a = W.p.a;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int e = blockIdx.y;
  const int ldc = cfg.ldc;
  const bool need = c < cfg.num_chains && entry_needed(cfg, a, c, e);
  if (!__syncthreads_or(need)) return;
  float s = 0.0f;
  if (need) {
    if (e == NPART) {
      for (int sl = wv; sl < W.ns; sl += WIDE_SWAVES) s += a.part0[(size_t)sl * ldc + c];
    } else {
      for (int sl = wv; sl < W.ns; sl += WIDE_SWAVES) s += *(part_ptr(a, ldc, sl, e) + c);
    }
  }
  lds[wv * 64 + lane] = s;
  __syncthreads();
  if (wv == 0 && need) {
    float t = 0.0f;
#pragma unroll
    for (int w = 0; w < WIDE_SWAVES; ++w) t += lds[w * 64 + lane];
    a.tot[(size_t)e * ldc + c] = t;
  }
}

// Scalar logic of the wide step, one wave per 64 chains, on the reduced totals.
__global__ __launch_bounds__(64) void k_wide_s(WideArgs W) {
  const nmx_nuts_config& cfg = W.p.cfg;
  const Arena& a = W.p.a;
  const int lane = threadIdx.x;
  const int c = blockIdx.x * 64 + lane;
  const int ldc = cfg.ldc;
  const bool valid = c < cfg.num_chains;
  const uint32_t gch = (uint32_t)(cfg.chain_offset + c);
  const uint64_t seed = cfg.seed;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.counters[2 + (cfg.parity ^ 1)] = 0;

  ChainScalars S;
  Act A;
  begin_step(cfg, a, c, valid, S, A);
  const int ph_in = S.phase;  // the stored phase (begin_step's return resolves WAIT)
  const bool ke0_pending = valid && (AI(NMX_F_ACTION)[c] & ACT_KE0_PENDING);
  const float* T = a.tot + c;
  if (ke0_pending) {
    S.E0 = S.pe + 0.5f * T[(size_t)NPART * ldc];  // build_tree :1130 (momentum KE from the last V2)
    S.energy = S.E0;
  }
  leaf_phase(cfg, S, A, A.leaf ? 0.5f * T[0] : 0.0f, seed, gch);
  tree_phase(
      cfg, S, A, [&](int i, int side) { return T[(size_t)(1 + 2 * i + side) * ldc]; },
      [&](int side) { return T[(size_t)(1 + 2 * MAXD + side) * ldc]; }, seed, gch, W.p.fields, c, true);
  if (valid) {
    AI(NMX_F_ACTION)[c] = pack_act(A);
    AI(NMX_F_SLOT)[c] = A.slot;
    AI(NMX_F_ACT_WFN)[c] = A.wfn;
  }
  // (a chain with ke0_pending is a LEAF chain, so end_step stores its E0)
  end_step(cfg, a, c, valid, ph_in, S, A);
}

#ifndef NMX_V2_WAVES
#define NMX_V2_WAVES 4
#endif
#ifndef NMX_V2_BATCH
#define NMX_V2_BATCH 2
#endif
constexpr int V2_WAVES = NMX_V2_WAVES;  // waves per V2 block: each takes momentum blocks wv, wv + V2_WAVES, ...

__global__ __launch_bounds__(64 * V2_WAVES) void k_wide_v2(WideArgs W) {
  __shared__ float lds[V2_WAVES * 64];
  const nmx_nuts_config& cfg = W.p.cfg;
  const Arena& a = W.p.a;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int s = blockIdx.y;
  const int ldc = cfg.ldc, D = cfg.dim;
  const bool valid = c < cfg.num_chains;
  // all per-chain scalars in one round of loads, ahead of the early exit (as in V1)
  int act = 0, slot = -1, wfn = 0, it = 0;
  float step_eff = 0.0f;
  if (valid) {
    act = AI(NMX_F_ACTION)[c];
    slot = AI(NMX_F_SLOT)[c];
    wfn = AI(NMX_F_ACT_WFN)[c];
    step_eff = AF(NMX_F_STEP_EFF)[c];
    it = AI(NMX_F_ITER)[c];
  }
  constexpr int VEC = ACT_TAKE_LEAF | ACT_DONE_SUB | ACT_TAKE_BIASED | ACT_HMC_ACCEPT | ACT_ITER_DONE | ACT_START |
                      ACT_PREP;
  if (!__syncthreads_or((act & VEC) != 0)) return;
  Act A{};
  A.take_leaf = act & ACT_TAKE_LEAF;
  A.done_sub = act & ACT_DONE_SUB;
  A.take_biased = act & ACT_TAKE_BIASED;
  A.hmc_accept = act & ACT_HMC_ACCEPT;
  A.iter_done = act & ACT_ITER_DONE;
  A.wf_update = act & ACT_WF_UPDATE;
  A.finalize = act & ACT_FINALIZE;
  A.start_iter = act & ACT_START;
  A.prep_leaf = act & ACT_PREP;
  A.dirR = (act & ACT_DIRR) ? 1 : 0;
  A.new_dir = (act & ACT_NEWDIR) ? 1 : 0;
  A.slot = slot;
  A.wfn = wfn;
  const uint32_t gch = (uint32_t)(cfg.chain_offset + c);
  float* const samp = (A.iter_done && A.slot >= 0 && W.p.samples) ? W.p.samples + (size_t)A.slot * D * ldc
                                                                   : nullptr;
  const VecCtx v{&a, ldc, D, (size_t)D * ldc, cfg.unit_mass != 0};
  float ke0[1] = {0.0f};
  if (act & VEC) {
    const int b0 = (s * W.sw) / 4, b1 = (min(D, (s + 1) * W.sw) + 3) / 4;
    for (int blk = b0 + wv; blk < b1; blk += V2_WAVES) {
      float n[4] = {0.f, 0.f, 0.f, 0.f};
      if (A.start_iter) momentum_block(cfg.seed, gch, it, blk, n);
      // rows in pairs: 95 VGPRs, 5 waves per SIMD (all four rows' loads first: 121 VGPRs, 4
      // waves; SV 1024 chains 3.58M vs 3.93M leapfrog/s, funnel-10k diag 658k vs 717k)
      ke0[0] += apply_block<NMX_V2_BATCH>(v, A, step_eff, blk, c, n, samp, W.p.transform, cfg);
    }
  }
  block_sum<V2_WAVES, 1>(ke0, lds);
  if (wv == 0 && A.start_iter) a.part0[(size_t)s * ldc + c] = ke0[0];
}

// ---- fused leaf of the wide schedule for the D-split models (nmx_wide_models.h) -----------
// The launched wide path runs six kernels per leaf: the model's part + fin, then V1, R, S, V2.
// For a model whose potential is per-row terms plus global sums, three suffice:
//   B  k_wide_leaf  (chain groups x D-slices): the model's row gradients and partial sums, with
//                   the leapfrog end (V1) of the same rows on the gradient in registers;
//   C  k_wide_rs    (chain groups x entries):  the fixed-order slice reduction of each partial
//                   entry (R); the last block of a chain group to finish then completes the
//                   potential (U and the scalar-site gradients), the leapfrog end of the
//                   scalar-site rows, and runs the scalar logic (S);
//   A  k_wide_v2    as before.
// Sums are in a fixed order that depends on D only (slices in order, scalar-site rows last),
// so draws stay independent of the launch composition and the number of GPUs; they differ
// from the six-kernel path in rounding only (the potential's slices are the step's here).
// Workspace: model partials [NS][WIDE_NSUM][ldc] f32, model totals [WIDE_NSUM][ldc] f32, one
// arrival counter per chain group (zero on entry; the last block leaves it zero).
constexpr int WIDE_NSUM = 4;  // largest M::NSUM


inline size_t wide_ws_part_bytes(int D, int ldc) { return align_up((size_t)num_slices(D) * WIDE_NSUM * ldc * 4); }
inline size_t wide_ws_tot_bytes(int ldc) { return align_up((size_t)WIDE_NSUM * ldc * 4); }

// NUTS leapfrog end of rows d0, d0 + step, ... < d1 with the model's gradient, one row per
// round: the row's leaf-state loads, then the model's loads (z and stencil neighbours), then
// the stores (the one-pass form of leaf_rows; same sums in the same order).  One row per round
// keeps k_wide_leaf at 168 VGPRs, 3 waves per SIMD: SV 1024 chains 3.57-3.58M vs 3.40M leapfrog/s
// with rows in pairs (229 VGPRs, 2 waves per SIMD), funnel-10k diag 657k vs 638k.
template <bool NUTS, class M>
__device__ __forceinline__ void leaf_rows_model(const VecCtx& v, const Act& A, const M& m, const typename M::Glob& gl,
                                                float seff, int d0, int d1, int step, int c, float* red,
                                                float* sums) {
  const Arena& a = *v.a;
  const float* ZE = AV(NMX_F_Z_EVAL);
  float* GE = AV(NMX_F_G_EVAL);
  int d = d0;
  const uint32_t ldc4 = (uint32_t)v.ldc << 2;
#ifndef NMX_LEAF_PIPE
#define NMX_LEAF_PIPE 0
#endif
  if constexpr (NMX_LEAF_PIPE) {
    // software-pipelined as leaf_rows<ROWS = 3>: the next row's leaf state and model inputs
    // are loaded before this row's model arithmetic and stores
    if (d >= d1) return;
    LeafIn cur;
    typename M::RowIn mc;
    uint32_t ic = nmx_row_off(d, v.ldc, c);
    leaf_load<NUTS, true, false>(v, A, ic, cur);
    m.row_load(ZE, ic, ldc4, d, mc);
    for (; d < d1; d += step) {
      const int dn = d + step;
      const uint32_t in = nmx_row_off(dn, v.ldc, c);
      LeafIn nxt;
      typename M::RowIn mn;
      if (dn < d1) {
        leaf_load<NUTS, true, false>(v, A, in, nxt);
        m.row_load(ZE, in, ldc4, dn, mn);
      }
      cur.g = m.row_eval(mc, d, gl, sums);
      nmx_at(GE, ic) = cur.g;
      leaf_store<NUTS, true>(v, A, seff, ic, cur, red);
      cur = nxt;
      mc = mn;
      ic = in;
    }
    return;
  }
  for (; d < d1; d += step) {
    const uint32_t i0 = nmx_row_off(d, v.ldc, c);
    LeafIn x0;
    leaf_load<NUTS, true, false>(v, A, i0, x0);
    x0.g = m.row(ZE, i0, ldc4, d, gl, sums);
    nmx_at(GE, i0) = x0.g;
    leaf_store<NUTS, true>(v, A, seff, i0, x0, red);
  }
}

#ifndef NMX_LEAF_OCC
#define NMX_LEAF_OCC 3  // waves per SIMD k_wide_leaf is compiled for (4: <= 128 VGPRs, small spills, slower)
#endif
template <class M>
__global__ __launch_bounds__(64 * WIDE_WAVES, NMX_LEAF_OCC) void k_wide_leaf(WideArgs W, M m, float* ppart) {
  constexpr int NR = NPART + M::NSUM;
  constexpr int WV = WIDE_WAVES;
  __shared__ float lds[NR * WV * 64];
  const nmx_nuts_config& cfg = W.p.cfg;
  const Arena& a = W.p.a;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int s = blockIdx.y;
  const int ldc = cfg.ldc, D = cfg.dim;
  const bool valid = c < cfg.num_chains;
  int ph = NMX_PH_DONE, dir = 0, subn = 0, depth = 0;
  float seff0 = 0.0f;
  if (valid) {
    ph = AI(NMX_F_PHASE)[c];
    dir = AI(NMX_F_DIR)[c];
    subn = AI(NMX_F_SUB_N)[c];
    depth = AI(NMX_F_DEPTH)[c];
    seff0 = AF(NMX_F_STEP_EFF)[c];
  }
  if (!__syncthreads_or(ph == NMX_PH_LEAF)) return;
  const bool is_nuts = cfg.algo == NMX_ALGO_NUTS;
  Act A{};
  A.leaf = ph == NMX_PH_LEAF;
  A.dirR = A.leaf ? dir : 0;
  A.k = (A.leaf && is_nuts) ? subn : 0;
  A.j = (A.leaf && is_nuts) ? depth : 0;
  A.imin = 1;
  A.imax = 0;
  if (A.leaf && is_nuts) nmx_leaf_idx_to_ckpt_idxs(A.k, A.imin, A.imax);
  A.tree_chk = A.leaf && is_nuts && (A.k + 1 == (1 << A.j));
  const float seff = A.leaf ? seff0 : 0.0f;
  const VecCtx v{&a, ldc, D, (size_t)D * ldc, cfg.unit_mass != 0};
  float red[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) red[i] = 0.0f;
  const int r0 = max(s * W.sw, m.lo()), r1 = min(min(D, (s + 1) * W.sw), m.hi());
  if (A.leaf) {
    const typename M::Glob gl = m.globals(AV(NMX_F_Z_EVAL), ldc, c);
    if (is_nuts) leaf_rows_model<true>(v, A, m, gl, seff, r0 + wv, r1, WV, c, red, red + NPART);
    else leaf_rows_model<false>(v, A, m, gl, seff, r0 + wv, r1, WV, c, red, red + NPART);
  }
  block_sum<WV, NR>(red, lds);
  if (wv == 0 && A.leaf) {
    *(part_ptr(a, ldc, s, 0) + c) = red[0];
    if (is_nuts) {
#pragma unroll
      for (int i = 0; i < MAXD; ++i)
        if (i >= A.imin && i <= A.imax) {
          *(part_ptr(a, ldc, s, 1 + 2 * i) + c) = red[1 + 2 * i];
          *(part_ptr(a, ldc, s, 2 + 2 * i) + c) = red[2 + 2 * i];
        }
      if (A.tree_chk) {
        *(part_ptr(a, ldc, s, 1 + 2 * MAXD) + c) = red[1 + 2 * MAXD];
        *(part_ptr(a, ldc, s, 2 + 2 * MAXD) + c) = red[2 + 2 * MAXD];
      }
    }
#pragma unroll
    for (int k = 0; k < M::NSUM; ++k) ppart[((size_t)s * WIDE_NSUM + k) * ldc + c] = red[NPART + k];
  }
}

// Reduction + (last block per chain group) potential finish, scalar-site leapfrog ends and
// scalar logic.  Entries 0..NPART-1 = V1 partials, NPART = momentum KE, NPART + 1 + k = the
// model's sum k.  The hand-off to the last block is the in-launch split reduction of
// cdna_hip_programming.md §6 G16: write-through (sc1) stores of the totals, every storing
// wave drained, a workgroup barrier, one relaxed agent-scope arrival add per block; the block
// drawing the last ticket acquires (agent) before reading them.
template <class M>
__global__ __launch_bounds__(64 * WIDE_SWAVES) void k_wide_rs(WideArgs W, M m, const float* ppart, float* ptot,
                                                            int* cnt) {
  constexpr int NE = NPART + 1 + M::NSUM;
  __shared__ float lds[WIDE_SWAVES * 64];
  __shared__ int last_block;
  const nmx_nuts_config& cfg = W.p.cfg;
  const Arena& a = W.p.a;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int e = blockIdx.y;
  const int ldc = cfg.ldc;
  const bool valid = c < cfg.num_chains;
  const int ph = valid ? AI(NMX_F_PHASE)[c] : NMX_PH_DONE;
  // every block of a chain group sees the same phases: a group with no live chain is skipped
  // by all of them (no arrival, no scalar logic: a DONE chain's step is a no-op)
  if (!__syncthreads_or(ph != NMX_PH_DONE)) return;
  bool need = false;
  if (valid) need = e <= NPART ? entry_needed(cfg, a, c, e) : ph == NMX_PH_LEAF;
  float sum = 0.0f;
  if (need) {
    if (e < NPART) {
      for (int sl = wv; sl < W.ns; sl += WIDE_SWAVES) sum += *(part_ptr(a, ldc, sl, e) + c);
    } else if (e == NPART) {
      for (int sl = wv; sl < W.ns; sl += WIDE_SWAVES) sum += a.part0[(size_t)sl * ldc + c];
    } else {
      const int k = e - NPART - 1;
      for (int sl = wv; sl < W.ns; sl += WIDE_SWAVES) sum += ppart[((size_t)sl * WIDE_NSUM + k) * ldc + c];
    }
  }
  lds[wv * 64 + lane] = sum;
  __syncthreads();
  if (wv == 0 && need) {
    float t = 0.0f;
#pragma unroll
    for (int w = 0; w < WIDE_SWAVES; ++w) t += lds[w * 64 + lane];
    float* dst = e <= NPART ? a.tot + (size_t)e * ldc + c : ptot + (size_t)(e - NPART - 1) * ldc + c;
    __hip_atomic_store(dst, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int ticket = __hip_atomic_fetch_add(&cnt[blockIdx.x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    NMX_DCHECK(ticket >= 0 && ticket < NE);  // the counters start at zero and are left at zero
    last_block = ticket == NE - 1;
  }
  __syncthreads();
  if (!last_block) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&cnt[blockIdx.x], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (wv != 0) return;

  // ---- last block, wave 0: one lane per chain ----
  const uint32_t gch = (uint32_t)(cfg.chain_offset + c);
  const uint64_t seed = cfg.seed;
  ChainScalars S;
  Act A;
  const int ph_in = ph;
  begin_step(cfg, a, c, valid, S, A);
  const bool ke0_pending = valid && (AI(NMX_F_ACTION)[c] & ACT_KE0_PENDING);
  const float* T = a.tot + c;
  if (ke0_pending) {
    S.E0 = S.pe + 0.5f * T[(size_t)NPART * ldc];  // build_tree :1130 (momentum KE from the last V2)
    S.energy = S.E0;
  }
  float red[NPART];
#pragma unroll
  for (int i = 0; i < NPART; ++i) red[i] = 0.0f;
  if (A.leaf) {
    // potential: U and the scalar-site gradients from the reduced sums
    float sums[M::NSUM];
#pragma unroll
    for (int k = 0; k < M::NSUM; ++k) sums[k] = ptot[(size_t)k * ldc + c];
    const typename M::Glob gl = m.globals(AV(NMX_F_Z_EVAL), ldc, c);
    float gs[M::NSCALAR];
    A.pe_eval = m.fin(sums, gl, gs);
    AF(NMX_F_PE_EVAL)[c] = A.pe_eval;
    // leapfrog end of the scalar-site rows (their partial dots join the totals last)
    const VecCtx v{&a, ldc, cfg.dim, (size_t)cfg.dim * ldc, cfg.unit_mass != 0};
    const bool is_nuts = cfg.algo == NMX_ALGO_NUTS;
#pragma unroll
    for (int i = 0; i < M::NSCALAR; ++i) {
      const uint32_t idx = nmx_row_off(m.scalar_row(i), ldc, c);
      nmx_at(AV(NMX_F_G_EVAL), idx) = gs[i];
      LeafIn x;
      x.g = gs[i];
      if (is_nuts) {
        leaf_load<true, true, false>(v, A, idx, x);
        leaf_store<true, true>(v, A, S.step_eff, idx, x, red);
      } else {
        leaf_load<false, true, false>(v, A, idx, x);
        leaf_store<false, true>(v, A, S.step_eff, idx, x, red);
      }
    }
  }
  leaf_phase(cfg, S, A, A.leaf ? 0.5f * (T[0] + red[0]) : 0.0f, seed, gch);
  tree_phase(
      cfg, S, A, [&](int i, int side) { return T[(size_t)(1 + 2 * i + side) * ldc] + red[1 + 2 * i + side]; },
      [&](int side) { return T[(size_t)(1 + 2 * MAXD + side) * ldc] + red[1 + 2 * MAXD + side]; }, seed, gch,
      W.p.fields, c, true);
  if (valid) {
    AI(NMX_F_ACTION)[c] = pack_act(A);
    AI(NMX_F_SLOT)[c] = A.slot;
    AI(NMX_F_ACT_WFN)[c] = A.wfn;
  }
  end_step(cfg, a, c, valid, ph_in, S, A, false);
}


// ---- persistent per-chain schedule for the D-split models ----------
// One workgroup of NT threads owns one chain (chain-row arena layout: the chain's rows are
// contiguous, so the threads' accesses coalesce) and runs its leaves until the segment ends or
// max_steps: the launched wide step's B / C / A kernels in one loop, with the chain's scalars
// in registers (every thread runs the scalar logic on block-reduced sums, as the fused step's
// lanes do; thread 0 writes).  Rows: thread t owns model rows lo + t, lo + t + NT, ... in both
// phases and thread 0 the scalar-site rows, so a row is read and written by one thread only
// within a leaf; the end-of-leaf barrier publishes the next positions (stencil neighbours and
// scalar sites) to the other threads.  Sums: per thread in row order, the 64 lanes of a wave
// by a butterfly, the waves in order, then the scalar-site rows -- fixed by (D, NT), NT by D.
// The scalar-site rows' inputs are staged through LDS before the reduction's barrier: every
// thread adds their terms to its totals, thread 0 alone stores them.

// sum over a wave's 64 lanes; the butterfly gives every lane the same bits
__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) x += __shfl_xor(x, o);
  return x;
}

// the partial-sum entries a leaf reduces (uniform over the block): KE, the checkpoint pairs of
// [imin, imax], the whole-tree pair at subtree completion, the model's sums (e >= NPART)
__device__ __forceinline__ bool entry_used(const Act& A, bool nuts, int e) {
  if (e == 0 || e >= NPART) return true;
  if (!nuts) return false;
  if (e >= 1 + 2 * MAXD) return A.tree_chk;
  const int i = (e - 1) >> 1;
  return i >= A.imin && i <= A.imax;
}

// stage 1 of the block sums: each wave's sum of every used entry -> lds[e * NW + wave]
template <int NW, int N>
__device__ __forceinline__ void wave_sums_to_lds(const float (&v)[N], float* lds, const Act& A, bool nuts) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int e = 0; e < N; ++e)
    if (entry_used(A, nuts, e)) {
      const float t = wave_sum(v[e]);
      if (lane == 0) lds[e * NW + wv] = t;
    }
}

// A row's leaf inputs in the persistent kernel: only the first U-turn checkpoint level [imin]
// is loaded with the row (the leaf_load arrays of all MAXD levels cost ~60 VGPRs at three rows
// in flight); leaves with more levels (a quarter of them) add one pass per extra level
// (persist_ckpt_levels).  Same arithmetic per row as leaf_load / leaf_store.
struct PRow {
  float rf, im, rs_old, rst, ro, ckr, ckrs;
};

// frontier momentum of row d: the LDS carry (CARRY) or the arena (byte offset off)
template <bool CARRY>
__device__ __forceinline__ float& front_r(const VecCtx& v, const Act& A, const Front& fr, uint32_t off, int d) {
  const Arena& a = *v.a;
  if constexpr (CARRY) return fr.r[d];
  else return nmx_at((A.dirR ? AV(NMX_F_RR) : AV(NMX_F_RL)), off);
}

template <bool NUTS, bool CARRY = false>
__device__ __forceinline__ void prow_load(const VecCtx& v, const Act& A, uint32_t off, PRow& x, const Front& fr = {},
                                          int d = 0) {
  const Arena& a = *v.a;
  x.rf = front_r<CARRY>(v, A, fr, off, d);
  x.im = v.unit ? 1.0f : (CARRY ? fr.im[d] : nmx_at(AV(NMX_F_INV_MASS), off));
  if constexpr (NUTS) {
    x.rs_old = A.k == 0 ? 0.0f : nmx_at(AV(NMX_F_RSUM_SUB), off);
    if (A.tree_chk) {
      x.rst = nmx_at(AV(NMX_F_RSUM), off);
      x.ro = nmx_at((A.dirR ? AV(NMX_F_RL) : AV(NMX_F_RR)), off);
    }
    if (A.imin <= A.imax) {
      x.ckr = nmx_at(a.ckr + A.imin * v.ck_stride, off);
      x.ckrs = nmx_at(a.ckrs + A.imin * v.ck_stride, off);
    }
  }
}

// red[0] KE, red[1 + 2 MAXD + side] tree dots; dl / dr: the dots of checkpoint level imin
// TL: the index of the tree dots in red (red[0] = KE): the full partial-sum vector's 1 + 2 MAXD,
// or 1 in the persistent kernel's compact accumulators (persist_leaf_rows)
template <bool NUTS, bool CARRY = false, int TL = 1 + 2 * MAXD>
__device__ __forceinline__ void prow_store(const VecCtx& v, const Act& A, float seff, uint32_t off, const PRow& x,
                                           float g, float* red, float& dl, float& dr, const Front& fr = {},
                                           int d = 0) {
  const Arena& a = *v.a;
  const float es = A.dirR ? seff : -seff;
  const float half = 0.5f * es;
  const float r = x.rf - half * g;
  front_r<CARRY>(v, A, fr, off, d) = r;
  const float im = x.im;
  red[0] += (im * r) * r;
  if constexpr (NUTS) {
    const float rs = (A.k == 0) ? r : x.rs_old + r;
    nmx_at(AV(NMX_F_RSUM_SUB), off) = rs;
    if ((A.k & 1) == 0) {  // checkpoint update (:1040-1047); even leaves read no checkpoint
      nmx_at(a.ckr + A.imax * v.ck_stride, off) = r;
      nmx_at(a.ckrs + A.imax * v.ck_stride, off) = rs;
    }
    if (A.imin <= A.imax) {
      const float rl = x.ckr;
      const float rsub = (rs - x.ckrs) + rl;
      const float rss = rsub - (rl + r) / 2.0f;  // _momentum_angle :735
      dl += (im * rl) * rss;
      dr += (im * r) * rss;
    }
    if (A.tree_chk) {
      const float rst = x.rst + rs;
      const float rlv = A.dirR ? x.ro : r;
      const float rrv = A.dirR ? r : x.ro;
      const float rss2 = rst - (rlv + rrv) / 2.0f;
      red[TL] += (im * rlv) * rss2;
      red[TL + 1] += (im * rrv) * rss2;
    }
  }
}

// The carry form's leaf rows: the frontier momentum, inverse mass and positions are LDS reads,
// so a row's HBM loads (subtree r_sum, the first checkpoint level, the tree's r_sum and other
// end at subtree completion, the model's data) are all that must be in flight across a batch:
// BC rows' worth of them go out first, then each row reads its LDS inputs and runs.  Five floats
// per row in flight instead of the arena form's eleven: larger batches fit the registers, fewer
// dependent memory rounds per leaf.  Same arithmetic as persist_leaf_rows.
// A thread's first model row, recomputed at each use: hoisted out of the leaf loop (as a 64-bit
// induction start) it was spilled, and its scratch reload before the apply loop put an
// s_waitcnt vmcnt(0) at the loop's back edge -- every apply row then waited for its own stores.
template <class M>
__device__ __forceinline__ int first_row(const M& m) {
  int d0 = m.lo() + (int)threadIdx.x;
  asm volatile("" : "+v"(d0));
  return d0;
}

#ifndef NMX_PX_PIPE
// persist_leaf_rows_carry software-pipelined over two batches (A/B: 55.6-56.1M with two buffers of
// 2 rows vs 57.2-57.5M unpipelined at SV 8192 chains -- the other chains' waves already cover the
// store drain; profiles/r06/sv_phase_stamps.txt)
#define NMX_PX_PIPE 0
#endif
#ifndef NMX_PX_BC
// rows per batch of the carry form's leaf rows: SV 8192 chains 2 / 3 / 4 rows 40.0 / 40.0 / 40.3M
// (before the apply loop's fix), 3 / 4 / 5: 42.5 / 42.7 / 42.8M (profiles/r06/sv_phase_stamps.txt)
#define NMX_PX_BC 4
#endif
struct PRowG {
  float rs_old, rst, ro, ckr, ckrs;
};
template <bool NUTS, int NT, int BC, class M>
__device__ __forceinline__ void persist_leaf_rows_carry(const VecCtx& v, const Act& A, const M& m,
                                                        const typename M::Glob& gl, float seff, uint32_t base,
                                                        float* red, const Front& fr) {
  const Arena& a = *v.a;
  const int hi = m.hi();
  float dl = 0.0f, dr = 0.0f;
  float acc[3 + M::NSUM];
#pragma unroll
  for (int i = 0; i < 3 + M::NSUM; ++i) acc[i] = 0.0f;
  // a batch's loads, grouped by their (wave-uniform) condition, every row of the batch included: a
  // row past hi reads row hi - 1 (a valid address; the value is never used).  Per-row guards around
  // the loads split them into small blocks, and the compiler drained the first row's loads
  // (s_waitcnt vmcnt(0)) before issuing the rest.
  auto load = [&](int d0, PRowG (&xg)[BC], typename M::RowIn (&mi)[BC]) {
    uint32_t offq[BC];
#pragma unroll
    for (int q = 0; q < BC; ++q) {
      const int d = min(d0 + q * NT, hi - 1);
      offq[q] = base + ((uint32_t)d << 2);
      m.row_load_data(d, mi[q]);
    }
    if constexpr (NUTS) {
      if (A.k != 0) {
#pragma unroll
        for (int q = 0; q < BC; ++q) xg[q].rs_old = nmx_at(AV(NMX_F_RSUM_SUB), offq[q]);
      } else {
#pragma unroll
        for (int q = 0; q < BC; ++q) xg[q].rs_old = 0.0f;
      }
      if (A.tree_chk) {
        const float* RO = A.dirR ? AV(NMX_F_RL) : AV(NMX_F_RR);
#pragma unroll
        for (int q = 0; q < BC; ++q) {
          xg[q].rst = nmx_at(AV(NMX_F_RSUM), offq[q]);
          xg[q].ro = nmx_at(RO, offq[q]);
        }
      }
      if (A.imin <= A.imax) {
        const float* CK = a.ckr + A.imin * v.ck_stride;
        const float* CKS = a.ckrs + A.imin * v.ck_stride;
#pragma unroll
        for (int q = 0; q < BC; ++q) {
          xg[q].ckr = nmx_at(CK, offq[q]);
          xg[q].ckrs = nmx_at(CKS, offq[q]);
        }
      }
    }
  };
  auto compute = [&](int d0, const PRowG (&xg)[BC], typename M::RowIn (&mi)[BC]) {
#pragma unroll
    for (int q = 0; q < BC; ++q) {
      const int d = d0 + q * NT;
      if (d < hi) {
        const uint32_t off = base + ((uint32_t)d << 2);
        PRow x;
        x.rf = fr.r[d];
        x.im = v.unit ? 1.0f : fr.im[d];
        x.rs_old = xg[q].rs_old;
        x.rst = xg[q].rst;
        x.ro = xg[q].ro;
        x.ckr = xg[q].ckr;
        x.ckrs = xg[q].ckrs;
        m.row_load_z(fr.z, (uint32_t)d << 2, 4u, d, mi[q]);  // stencil neighbours too
        const float g = m.row_eval(mi[q], d, gl, acc + 3);
        fr.g[d] = g;
        prow_store<NUTS, true, 1>(v, A, seff, off, x, g, acc, dl, dr, fr, d);
      }
    }
  };
#if NMX_PX_PIPE
  // software-pipelined over two register buffers: batch b + 1's loads go out before batch b's
  // stores, so the wait for them does not also wait for those stores (loads and stores share
  // vmcnt, in order) -- one batch per memory round instead of a full store drain per batch
  PRowG xa[BC], xb[BC];
  typename M::RowIn ma[BC], mb[BC];
  int d0 = first_row(m);
  if (d0 < hi) load(d0, xa, ma);
  while (d0 < hi) {
    int d1 = d0 + BC * NT;
    if (d1 < hi) load(d1, xb, mb);
    compute(d0, xa, ma);
    d0 = d1;
    if (d0 >= hi) break;
    d1 = d0 + BC * NT;
    if (d1 < hi) load(d1, xa, ma);
    compute(d0, xb, mb);
    d0 = d1;
  }
#else
  for (int d0 = first_row(m); d0 < hi; d0 += BC * NT) {
    PRowG xg[BC];
    typename M::RowIn mi[BC];
    load(d0, xg, mi);
    compute(d0, xg, mi);
  }
#endif
  red[0] += acc[0];
  red[1 + 2 * MAXD] += acc[1];
  red[2 + 2 * MAXD] += acc[2];
#pragma unroll
  for (int k = 0; k < M::NSUM; ++k) red[NPART + k] += acc[3 + k];
  if constexpr (NUTS) {
#pragma unroll
    for (int i = 0; i < MAXD; ++i)
      if (i == A.imin && A.imin <= A.imax) {
        red[1 + 2 * i] = dl;
        red[2 + 2 * i] = dr;
      }
  }
}

template <bool NUTS, int NT, int B, bool CARRY, class M>
__device__ __forceinline__ void persist_leaf_rows(const VecCtx& v, const Act& A, const M& m,
                                                  const typename M::Glob& gl, float seff, uint32_t base, float* red,
                                                  const Front& fr) {
  const Arena& a = *v.a;
  const float* ZE = AV(NMX_F_Z_EVAL);
  float* GE = AV(NMX_F_G_EVAL);
  const int hi = m.hi();
  float dl = 0.0f, dr = 0.0f;
  // compact accumulators through the row loop (KE, the tree dots, the model's sums: the unused
  // checkpoint entries of red stay out of the registers), expanded into red after it
  float acc[3 + M::NSUM];
#pragma unroll
  for (int i = 0; i < 3 + M::NSUM; ++i) acc[i] = 0.0f;
  for (int d0 = first_row(m); d0 < hi; d0 += B * NT) {
    PRow x[B];
    typename M::RowIn mi[B];
#pragma unroll
    for (int q = 0; q < B; ++q) {
      const int d = d0 + q * NT;
      if (d < hi) {
        const uint32_t off = base + ((uint32_t)d << 2);
        prow_load<NUTS, CARRY>(v, A, off, x[q], fr, d);
        if constexpr (CARRY) m.row_load(fr.z, (uint32_t)d << 2, 4u, d, mi[q]);  // stencil neighbours too
        else m.row_load(ZE, off, 4u, d, mi[q]);
      }
    }
#pragma unroll
    for (int q = 0; q < B; ++q) {
      const int d = d0 + q * NT;
      if (d < hi) {
        const uint32_t off = base + ((uint32_t)d << 2);
        const float g = m.row_eval(mi[q], d, gl, acc + 3);
        if constexpr (CARRY) fr.g[d] = g;
        else nmx_at(GE, off) = g;
        prow_store<NUTS, CARRY, 1>(v, A, seff, off, x[q], g, acc, dl, dr, fr, d);
      }
    }
  }
  red[0] += acc[0];
  red[1 + 2 * MAXD] += acc[1];
  red[2 + 2 * MAXD] += acc[2];
#pragma unroll
  for (int k = 0; k < M::NSUM; ++k) red[NPART + k] += acc[3 + k];
  if constexpr (NUTS) {
#pragma unroll
    for (int i = 0; i < MAXD; ++i)
      if (i == A.imin && A.imin <= A.imax) {
        red[1 + 2 * i] = dl;
        red[2 + 2 * i] = dr;
      }
  }
}

// U-turn dots of checkpoint levels imin + 1 .. imax (after wave_sums_to_lds): one pass over the
// thread's model rows per level, reloading the momentum / r_sum this leaf stored; each level's
// wave sums go straight to its LDS entries.
template <int NW, int NT, bool CARRY = false, class M>
__device__ __forceinline__ void persist_ckpt_levels(const VecCtx& v, const Act& A, const M& m, uint32_t base,
                                                    float* lds, const Front& fr = {}) {
  constexpr int B2 = 4;
  const Arena& a = *v.a;
  const float* RF = A.dirR ? AV(NMX_F_RR) : AV(NMX_F_RL);
  const float* RS = AV(NMX_F_RSUM_SUB);
  const float* IM = AV(NMX_F_INV_MASS);
  const int hi = m.hi();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int i = A.imin + 1; i <= A.imax; ++i) {
    const float* CK = a.ckr + i * v.ck_stride;
    const float* CKS = a.ckrs + i * v.ck_stride;
    float dl = 0.0f, dr = 0.0f;
    for (int d0 = first_row(m); d0 < hi; d0 += B2 * NT) {
      float r[B2], rs[B2], im[B2], rl[B2], rls[B2];
#pragma unroll
      for (int q = 0; q < B2; ++q) {
        const int d = d0 + q * NT;
        if (d < hi) {
          const uint32_t off = base + ((uint32_t)d << 2);
          if constexpr (CARRY) r[q] = fr.r[d];
          else r[q] = nmx_at(RF, off);
          rs[q] = nmx_at(RS, off);
          im[q] = v.unit ? 1.0f : (CARRY ? fr.im[d] : nmx_at(IM, off));
          rl[q] = nmx_at(CK, off);
          rls[q] = nmx_at(CKS, off);
        }
      }
#pragma unroll
      for (int q = 0; q < B2; ++q) {
        if (d0 + q * NT < hi) {
          const float rsub = (rs[q] - rls[q]) + rl[q];
          const float rss = rsub - (rl[q] + r[q]) / 2.0f;
          dl += (im[q] * rl[q]) * rss;
          dr += (im[q] * r[q]) * rss;
        }
      }
    }
    const float tl = wave_sum(dl), tr = wave_sum(dr);
    if (lane == 0) {
      lds[(1 + 2 * i) * NW + wv] = tl;
      lds[(2 + 2 * i) * NW + wv] = tr;
    }
  }
}

// apply rows of thread t (model rows as in the leaf phase, then thread 0's scalar-site rows)
template <int NT, int B, bool CARRY = false, class M>
__device__ __forceinline__ float persist_apply_rows(const VecCtx& v, const Act& A, const M& m, float step_eff,
                                                   uint32_t base, int c, uint64_t seed, uint32_t gch, int it,
                                                   float* samp, const int8_t* transform,
                                                   const nmx_nuts_config& cfg, const Front& fr = {}) {
  float ke0 = 0.0f;
  const int hi = m.hi();
  auto rows = [&](int d0, int dstep, int dend, auto bc) {
    constexpr int BB = decltype(bc)::value;
    for (; d0 < dend; d0 += BB * dstep) {
      ApplyIn x[BB];
      float n[BB];
#pragma unroll
      for (int q = 0; q < BB; ++q) {
        const int d = d0 + q * dstep;
        if (d < dend) apply_load<CARRY>(v, A, base + ((uint32_t)d << 2), x[q], fr, d);
      }
#pragma unroll
      for (int q = 0; q < BB; ++q) {
        const int d = d0 + q * dstep;
        n[q] = 0.0f;
        if (A.start_iter && d < dend) {
          float nb[4];
          momentum_block(seed, gch, it, d >> 2, nb);
          const int j = d & 3;
          n[q] = j == 0 ? nb[0] : (j == 1 ? nb[1] : (j == 2 ? nb[2] : nb[3]));
        }
      }
#pragma unroll
      for (int q = 0; q < BB; ++q) {
        const int d = d0 + q * dstep;
        if (d < dend)
          ke0 += apply_store<CARRY>(v, A, step_eff, d, base + ((uint32_t)d << 2), x[q], n[q], samp, transform, cfg,
                                    nmx_row_off(d, v.ldc, c), fr);
      }
    }
  };
  rows(first_row(m), NT, hi, std::integral_constant<int, B>{});
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < M::NSCALAR; ++i) {
      const int d = m.scalar_row(i);
      rows(d, 1, d + 1, std::integral_constant<int, 1>{});
    }
  }
  return ke0;
}


// The apply phase of a mid-trajectory leaf (CARRY): the next half step and position of the
// frontier (prep_leaf, no turn-around), the proposal copy when the leaf is taken, nothing else --
// apply_load / apply_store's arithmetic on the same values, without their rare branches.  In the
// general loop the rare branches' conditional arena loads were merged into selects on registers a
// previous row may still have been loading, and every row waited (s_waitcnt vmcnt(0)) for all
// stores in flight; this loop has no global load at all.
template <int NT, class M>
__device__ __forceinline__ void persist_apply_prep_rows(const VecCtx& v, const Act& A, const M& m, float step_eff,
                                                        uint32_t base, const Front& fr) {
  const Arena& a = *v.a;
  const float es = A.new_dir ? step_eff : -step_eff;
  const float half = 0.5f * es;
  auto row = [&](int d) {
    const float ze = fr.z[d], ge = fr.g[d];
    if (A.take_leaf) {
      const uint32_t off = base + ((uint32_t)d << 2);
      nmx_at(AV(NMX_F_ZSUB), off) = ze;
      nmx_at(AV(NMX_F_GSUB), off) = ge;
    }
    const float im = v.unit ? 1.0f : fr.im[d];
    const float rh = fr.r[d] - half * ge;
    fr.r[d] = rh;
    fr.z[d] = ze + es * (im * rh);
  };
  const int hi = m.hi();
  for (int d = first_row(m); d < hi; d += NT) row(d);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < M::NSCALAR; ++i) row(m.scalar_row(i));
  }
}

// The same mid-trajectory apply on the arena (k_chain_step, no LDS frontier): B rows' loads, then
// their stores -- apply_load / apply_store's prep-leaf arithmetic without the generic loop's merged
// rare-branch loads (each of its rows waited for every store in flight).
template <int NT, int B, class M>
__device__ __forceinline__ void apply_prep_rows_arena(const VecCtx& v, const Act& A, const M& m, float step_eff,
                                                      uint32_t base) {
  const Arena& a = *v.a;
  const float es = A.new_dir ? step_eff : -step_eff;
  const float half = 0.5f * es;
  const float* RF = A.new_dir ? AV(NMX_F_RR) : AV(NMX_F_RL);
  float* RW = A.new_dir ? AV(NMX_F_RR) : AV(NMX_F_RL);
  float* ZE = AV(NMX_F_Z_EVAL);
  const int hi = m.hi();
  for (int d0 = first_row(m); d0 < hi; d0 += B * NT) {
    float ze[B], ge[B], im[B], rf[B];
    uint32_t offq[B];
#pragma unroll
    for (int q = 0; q < B; ++q) {
      const int d = min(d0 + q * NT, hi - 1);  // past hi: row hi - 1, loaded and not used
      offq[q] = base + ((uint32_t)d << 2);
      ze[q] = nmx_at(ZE, offq[q]);
      ge[q] = nmx_at(AV(NMX_F_G_EVAL), offq[q]);
      im[q] = v.unit ? 1.0f : nmx_at(AV(NMX_F_INV_MASS), offq[q]);
      rf[q] = nmx_at(RF, offq[q]);
    }
#pragma unroll
    for (int q = 0; q < B; ++q) {
      if (d0 + q * NT < hi) {
        if (A.take_leaf) {
          nmx_at(AV(NMX_F_ZSUB), offq[q]) = ze[q];
          nmx_at(AV(NMX_F_GSUB), offq[q]) = ge[q];
        }
        const float rh = rf[q] - half * ge[q];
        nmx_at(RW, offq[q]) = rh;
        nmx_at(ZE, offq[q]) = ze[q] + es * (im[q] * rh);
      }
    }
  }
}

// wave-uniform copies of values every lane holds alike (LDS reads look divergent to the
// compiler; as scalars they stay out of the vector registers)
__device__ __forceinline__ int uni_i(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ float uni_f(float x) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}

// Leaf inputs of the scalar-site rows, prefetched into LDS by the last wave at the start of a
// leaf (one value per lane, written after its own rows), so that the potential's finish in
// wave 0 runs their leapfrog end without a memory round trip.  Entry f of row i: 0 momentum of
// the moving end, 1 inverse mass, 2 subtree r_sum, 3 tree r_sum, 4 the other end's momentum,
// 5 + l / 5 + MAXD + l checkpoint momentum / r_sum of level l.
constexpr int SPRE = 5 + 2 * MAXD;

__device__ __forceinline__ const float* spre_src(const VecCtx& v, const Act& A, bool nuts, int f) {
  const Arena& a = *v.a;
  if (f == 0) return A.dirR ? AV(NMX_F_RR) : AV(NMX_F_RL);
  if (f == 1) return v.unit ? nullptr : AV(NMX_F_INV_MASS);
  if (!nuts) return nullptr;
  if (f == 2) return A.k == 0 ? nullptr : AV(NMX_F_RSUM_SUB);
  if (f == 3) return A.tree_chk ? AV(NMX_F_RSUM) : nullptr;
  if (f == 4) return A.tree_chk ? (A.dirR ? AV(NMX_F_RL) : AV(NMX_F_RR)) : nullptr;
  const int l = f < 5 + MAXD ? f - 5 : f - 5 - MAXD;
  if (l < A.imin || l > A.imax) return nullptr;
  return (f < 5 + MAXD ? a.ckr : a.ckrs) + l * v.ck_stride;
}

// leaf_load + leaf_store of one scalar-site row from its prefetched inputs (same arithmetic)
template <bool NUTS, bool CARRY = false>
__device__ __forceinline__ void spre_leaf(const VecCtx& v, const Act& A, float seff, uint32_t off, float g,
                                          const float* pre, float* red, const Front& fr = {}, int d = 0) {
  const Arena& a = *v.a;
  const float es = A.dirR ? seff : -seff;
  const float half = 0.5f * es;
  const float r = pre[0] - half * g;
  front_r<CARRY>(v, A, fr, off, d) = r;
  const float im = v.unit ? 1.0f : pre[1];
  red[0] += (im * r) * r;
  if constexpr (NUTS) {
    const float rs = (A.k == 0) ? r : pre[2] + r;
    nmx_at(AV(NMX_F_RSUM_SUB), off) = rs;
    if ((A.k & 1) == 0) {
      nmx_at(a.ckr + A.imax * v.ck_stride, off) = r;
      nmx_at(a.ckrs + A.imax * v.ck_stride, off) = rs;
    }
#pragma unroll
    for (int i = 0; i < MAXD; ++i) {
      if (i >= A.imin && i <= A.imax) {
        const float rl = pre[5 + i];
        const float rsub = (rs - pre[5 + MAXD + i]) + rl;
        const float rss = rsub - (rl + r) / 2.0f;
        red[1 + 2 * i] += (im * rl) * rss;
        red[2 + 2 * i] += (im * r) * rss;
      }
    }
    if (A.tree_chk) {
      const float rst = pre[3] + rs;
      const float rlv = A.dirR ? pre[4] : r;
      const float rrv = A.dirR ? r : pre[4];
      const float rss2 = rst - (rlv + rrv) / 2.0f;
      red[1 + 2 * MAXD] += (im * rlv) * rss2;
      red[2 + 2 * MAXD] += (im * rrv) * rss2;
    }
  }
}

#ifndef NMX_PX_OCC
#define NMX_PX_OCC 4  // waves per SIMD the kernel is compiled for: <= 128 VGPRs (3 waves: SV 8192 20.0M vs 24.2M)
#endif
// k_wide_persistent's static LDS, one struct (no padding between arrays; persist_carry sizes the
// carry form's dynamic LDS by it).  lds: the leaf's wave sums.  The chain's scalar state lives in
// LDS: wave 0 runs the scalar logic on it and publishes the decisions the vector phases need
// (the act word of k_wide_v2 plus two values; the iteration and step size are the state's), so
// no per-chain scalar is held in vector registers through the row loops.  sep: the momentum KE
// wave sums, the scalar-site rows' terms, the block totals (entries, then U) and the prefetched
// scalar-site row inputs; the carry form, where every byte of the workgroup's LDS share counts,
// keeps the first three in lds itself (wave 0 writes them after its lanes read every wave sum;
// the KE sums after the scalar logic, with a barrier before the next leaf's wave sums) and the
// prefetched inputs in wave 0's registers.
// The persistent wide kernel's serial section (wave 0: the potential's finish and the NUTS
// scalar logic, while the chain's other waves wait at a barrier) runs at raised wave priority, so
// the SIMD's arbiter issues it ahead of the row work of the other chains' waves sharing the SIMD
// (their phases are throughput-bound; the serial section is the chain's critical path).
#ifndef NMX_PX_PRIO
#define NMX_PX_PRIO 1
#endif
__device__ __forceinline__ void nmx_serial_prio(bool on) {
#if NMX_PX_PRIO
  if (on) __builtin_amdgcn_s_setprio(3);
  else __builtin_amdgcn_s_setprio(0);
#endif
}

template <int NT, class M, bool CARRY>
struct PersistShared {
  static constexpr int NW = NT / 64, NR = NPART + M::NSUM;
  static constexpr int NL = (CARRY && NR + 1 + NPART + NW > NR * NW) ? NR + 1 + NPART + NW : NR * NW;
  float lds[NL];
  ChainScalars S;
  int act, slot, wfn;
  float sep[CARRY ? 1 : NW + NPART + NR + 1 + M::NSCALAR * SPRE];
};

// CARRY: the chain's frontier and inverse mass (Front) live in LDS for the whole launch (16 D
// bytes of dynamic LDS, within the occupancy the kernel is compiled for: persist_carry): per leaf
// and row the arena then sees the subtree r_sum, the U-turn checkpoints and the proposal copies,
// not the frontier's position, gradient and momentum (loaded at entry, written back at exit and
// at turn-arounds) nor the inverse mass, and the stencil reads its neighbours from LDS: a
// leaf's apply rows usually read nothing from HBM.  Same arithmetic, bitwise equal.
template <int NT, int B, class M, bool CARRY>
__global__ __launch_bounds__(NT, NMX_PX_OCC) void k_wide_persistent(StepArgs Pk, M m, int max_steps) {
  constexpr int NW = NT / 64;
  constexpr int NR = NPART + M::NSUM;
  // lds: the leaf's wave sums.  CARRY (every byte of the workgroup's LDS share counts: four
  // [D] vectors beside these arrays) keeps the block totals (lds_tot, NR + 1: the entries, then
  // U) and the scalar-site rows' terms (lds_sc) in lds itself -- wave 0 writes them after its
  // lanes read every wave sum -- and the scalar-site rows' prefetched inputs in wave 0's
  // registers instead of lds_pre
  __shared__ PersistShared<NT, M, CARRY> sh;
  float* const lds = sh.lds;
  ChainScalars& Ssh = sh.S;
  float* const lds_sc = CARRY ? lds + NR + 1 : sh.sep + NW;
  float* const lds_tot = CARRY ? lds : sh.sep + NW + NPART;  // block totals of the leaf's entries, then U
  float* const lds_ke = CARRY ? lds + NR + 1 + NPART : sh.sep;  // (a transition's start: barrier below)
  float* const lds_pre = CARRY ? nullptr : sh.sep + NW + NPART + NR + 1;  // prefetched scalar-site row inputs
  static_assert(M::NSCALAR * SPRE <= 64, "one lane per prefetched value");
  const StepArgs& P = Pk;
  const nmx_nuts_config& cfg = P.cfg;
  const Arena& a = P.a;
  const int c = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int D = cfg.dim, ldc = cfg.ldc;
  const bool is_nuts = cfg.algo == NMX_ALGO_NUTS;
  const uint32_t gch = (uint32_t)(cfg.chain_offset + c);
  const uint64_t seed = cfg.seed;
  if (uni_i(AI(NMX_F_PHASE)[c]) == NMX_PH_DONE) return;
  if (tid == 0) {
    ChainScalars S;
    load_scalars(a, c, S);
    NMX_DCHECK(S.phase == NMX_PH_START || S.phase == NMX_PH_LEAF);
    Ssh = S;
  }
  const uint32_t base = ((uint32_t)c * (uint32_t)D) << 2;  // byte offset of the chain's row 0
  extern __shared__ float front_lds[];
  const Front fr{front_lds, front_lds + D, front_lds + 2 * D, front_lds + 3 * D};
  if constexpr (CARRY) {
    // the frontier of the pending leaf (START: overwritten by the momentum draw before any use)
    const int dir0 = uni_i(AI(NMX_F_DIR)[c]);
    const float* ZE = AV(NMX_F_Z_EVAL);
    const float* GE = AV(NMX_F_G_EVAL);
    const float* RF = dir0 ? AV(NMX_F_RR) : AV(NMX_F_RL);
    const float* IM = AV(NMX_F_INV_MASS);
    const bool unit = cfg.unit_mass != 0;
    for (int d = tid; d < D; d += NT) {
      const uint32_t off = base + ((uint32_t)d << 2);
      fr.z[d] = nmx_at(ZE, off);
      fr.g[d] = nmx_at(GE, off);
      fr.r[d] = nmx_at(RF, off);
      fr.im[d] = unit ? 1.0f : nmx_at(IM, off);
    }
  }
  __syncthreads();
  for (int step = 0; step < max_steps; ++step) {
    // the field pointers are recomputed each leaf (cheap scalar arithmetic) rather than
    // hoisted out of the loop: ~40 loop-invariant 64-bit pointers overflowed the SGPRs
    Arena al = Pk.a;
    size_t ck_stride = (size_t)D * ldc;
#ifndef NMX_DEBUG  // (the debug build's checks leave some of them in VGPRs: no SGPR constraint there)
    pin_sgpr_global(al.sbase);
    pin_sgpr_global(al.vbase);
    pin_sgpr_global(al.ckr);
    pin_sgpr_global(al.ckrs);
    asm volatile("" : "+s"(al.sstride), "+s"(al.vstride));
    asm volatile("" : "+s"(ck_stride));
#endif
    const VecCtx v{&al, ldc, D, ck_stride, cfg.unit_mass != 0};
    const int ph = uni_i(Ssh.phase);
    if (ph == NMX_PH_DONE) break;
    // the leaf's inputs (begin_act on the four scalars it reads)
    Act A;
    {
      ChainScalars Sb;
      Sb.dir = uni_i(Ssh.dir);
      Sb.sub_n = uni_i(Ssh.sub_n);
      Sb.depth = uni_i(Ssh.depth);
      begin_act(cfg, Sb, ph, A);
    }
    // every wave has read the state before wave 0's scalar logic rewrites it (a leaf's
    // reduction barrier orders this too)
    if (!A.leaf) __syncthreads();
    if (A.leaf) {
      const float seff = uni_f(Ssh.step_eff);
      // the scalar-site rows' inputs are prefetched: by the last wave into lds_pre after its rows,
      // or (CARRY) by wave 0 into the register pv, read by its lane 0 in the potential's finish
      float pv = 0.0f;
      bool pl = false;
      if (wv == (CARRY ? 0 : NW - 1) && lane < M::NSCALAR * SPRE) {
        const int i = lane / SPRE, f = lane % SPRE;
        const float* src = spre_src(v, A, is_nuts, f);
        if (src) {
          const int d = m.scalar_row(i);
          pv = (CARRY && f == 0) ? fr.r[d] : (CARRY && f == 1) ? fr.im[d] : nmx_at(src, base + ((uint32_t)d << 2));
          pl = true;
        }
      }
      const typename M::Glob gl = CARRY ? m.globals_at(fr.z, 0u, 4u) : m.globals_at(AV(NMX_F_Z_EVAL), base, 4u);
      {
        float red[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) red[i] = 0.0f;
        if constexpr (CARRY) {
          if (is_nuts) persist_leaf_rows_carry<true, NT, NMX_PX_BC>(v, A, m, gl, seff, base, red, fr);
          else persist_leaf_rows_carry<false, NT, NMX_PX_BC>(v, A, m, gl, seff, base, red, fr);
        } else {
          if (is_nuts) persist_leaf_rows<true, NT, NMX_PX_BL, CARRY>(v, A, m, gl, seff, base, red, fr);
          else persist_leaf_rows<false, NT, NMX_PX_BL, CARRY>(v, A, m, gl, seff, base, red, fr);
        }
        wave_sums_to_lds<NW, NR>(red, lds, A, is_nuts);
      }
      if (is_nuts && A.imax > A.imin) persist_ckpt_levels<NW, NT, CARRY>(v, A, m, base, lds, fr);
      if (!CARRY && pl) lds_pre[lane] = pv;
      __syncthreads();
      if (wv == 0) {
        nmx_serial_prio(true);
        // lane e: entry e's total over the waves (in wave order)
        float tot = 0.0f;
        if (lane < NR && entry_used(A, is_nuts, lane)) {
#pragma unroll
          for (int w = 0; w < NW; ++w) tot += lds[lane * NW + w];
        }
        // potential: U and the scalar-site gradients from the reduced sums (every lane alike)
        float sums[M::NSUM];
#pragma unroll
        for (int k = 0; k < M::NSUM; ++k) sums[k] = __shfl(tot, NPART + k);
        float gs[M::NSCALAR];
        const float pe = m.fin(sums, gl, gs);
        // the scalar-site rows' leapfrog end (thread 0 owns them in both phases); their terms
        // join the totals after the rows'
        if (lane == 0) {
          float rs[NPART];
#pragma unroll
          for (int e = 0; e < NPART; ++e) rs[e] = 0.0f;
#pragma unroll
          for (int i = 0; i < M::NSCALAR; ++i) {
            const int d = m.scalar_row(i);
            const uint32_t off = base + ((uint32_t)d << 2);
            float prer[CARRY ? SPRE : 1];
            const float* pre;
            if constexpr (CARRY) {
#pragma unroll
              for (int f = 0; f < SPRE; ++f)
                prer[f] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pv), i * SPRE + f));
              pre = prer;
              fr.g[d] = gs[i];
            } else {
              pre = lds_pre + i * SPRE;
              nmx_at(AV(NMX_F_G_EVAL), off) = gs[i];
            }
            if (is_nuts) spre_leaf<true, CARRY>(v, A, seff, off, gs[i], pre, rs, fr, d);
            else spre_leaf<false, CARRY>(v, A, seff, off, gs[i], pre, rs, fr, d);
          }
#pragma unroll
          for (int e = 0; e < NPART; ++e)
            if (entry_used(A, is_nuts, e)) lds_sc[e] = rs[e];
          lds_tot[NR] = pe;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < NPART && entry_used(A, is_nuts, lane)) tot += lds_sc[lane];
        if (lane < NR) lds_tot[lane] = tot;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
    // scalar logic: wave 0 on the LDS state (lane 0 writes back)
    if (wv == 0) {
      nmx_serial_prio(true);
      ChainScalars S = Ssh;
      if (A.leaf) A.pe_eval = lds_tot[NR];
      leaf_phase(cfg, S, A, A.leaf ? 0.5f * lds_tot[0] : 0.0f, seed, gch);
      tree_phase(
          cfg, S, A, [&](int i, int side) { return lds_tot[1 + 2 * i + side]; },
          [&](int side) { return lds_tot[1 + 2 * MAXD + side]; }, seed, gch, P.fields, c, lane == 0);
      if (lane == 0) {
        Ssh = S;
        sh.act = pack_act(A);
        sh.slot = A.slot;
        sh.wfn = A.wfn;
        if (A.fin_done) atomicAdd(&a.counters[0], 1);
      }
      nmx_serial_prio(false);
    }
    __syncthreads();  // decisions published
    const int act = uni_i(sh.act);
    {
      Act D2{};
      D2.take_leaf = act & ACT_TAKE_LEAF;
      D2.done_sub = act & ACT_DONE_SUB;
      D2.take_biased = act & ACT_TAKE_BIASED;
      D2.hmc_accept = act & ACT_HMC_ACCEPT;
      D2.iter_done = act & ACT_ITER_DONE;
      D2.wf_update = act & ACT_WF_UPDATE;
      D2.finalize = act & ACT_FINALIZE;
      D2.start_iter = act & ACT_START;
      D2.prep_leaf = act & ACT_PREP;
      D2.dirR = (act & ACT_DIRR) ? 1 : 0;
      D2.new_dir = (act & ACT_NEWDIR) ? 1 : 0;
      D2.slot = uni_i(sh.slot);
      D2.wfn = uni_i(sh.wfn);
      constexpr int VEC = ACT_TAKE_LEAF | ACT_DONE_SUB | ACT_TAKE_BIASED | ACT_HMC_ACCEPT | ACT_ITER_DONE |
                          ACT_START | ACT_PREP;
      float ke0 = 0.0f;
      constexpr int RARE = ACT_DONE_SUB | ACT_TAKE_BIASED | ACT_HMC_ACCEPT | ACT_ITER_DONE | ACT_WF_UPDATE |
                           ACT_FINALIZE | ACT_START;
      if (CARRY && NMX_PX_FAST_APPLY && (act & ACT_PREP) && !(act & RARE) && D2.new_dir == D2.dirR) {
        persist_apply_prep_rows<NT>(v, D2, m, uni_f(Ssh.step_eff), base, fr);
      } else if (act & VEC) {
        float* const samp = (D2.iter_done && D2.slot >= 0 && P.samples) ? P.samples + (size_t)D2.slot * D * ldc
                                                                         : nullptr;
        ke0 = persist_apply_rows<NT, B, CARRY>(v, D2, m, uni_f(Ssh.step_eff), base, c, seed, gch, uni_i(Ssh.it), samp,
                                               P.transform, cfg, fr);
      }
      if (D2.start_iter) {
        const float t = wave_sum(ke0);
        if (lane == 0) lds_ke[wv] = t;
      }
      __syncthreads();  // this leaf's rows are written: the next leaf reads its neighbours' positions
      if (threadIdx.x == 0) {
      }
      if (D2.start_iter && tid == 0) {
        float t = 0.0f;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += lds_ke[w];
        Ssh.E0 = Ssh.pe + 0.5f * t;  // build_tree :1130
        Ssh.energy = Ssh.E0;         // proposal energy of the initial tree (:1137)
      }
      if (CARRY && D2.start_iter) __syncthreads();  // lds_ke read before the next leaf's wave sums
    }
  }
  if constexpr (CARRY) {
    // the frontier back to the arena (every thread passed the loop's last barrier: its LDS is final)
    const Arena& al = Pk.a;
    const int dir1 = uni_i(Ssh.dir);
    float* ZE = reinterpret_cast<float*>(al.vbase + (size_t)(NMX_F_Z_EVAL - NMX_F_Z) * al.vstride);
    float* GE = reinterpret_cast<float*>(al.vbase + (size_t)(NMX_F_G_EVAL - NMX_F_Z) * al.vstride);
    float* RF = reinterpret_cast<float*>(al.vbase + (size_t)((dir1 ? NMX_F_RR : NMX_F_RL) - NMX_F_Z) * al.vstride);
    for (int d = tid; d < D; d += NT) {
      const uint32_t off = base + ((uint32_t)d << 2);
      nmx_at(ZE, off) = fr.z[d];
      nmx_at(GE, off) = fr.g[d];
      nmx_at(RF, off) = fr.r[d];
    }
  }
  if (tid == 0) {
    Arena al = Pk.a;  // addresses recomputed here, not kept live from load_scalars through the loop
    pin_sgpr_global(al.sbase);
    asm volatile("" : "+s"(al.sstride));
    store_scalars(al, c, Ssh);
  }
}


// ---- launched per-chain step for a chain-row arena -------------------
// The D-split models behind a batched potential (dense mass: the whitening GEMMs couple the
// chains between leaves, so the persistent kernel does not apply) keep the launched loop, but
// its step runs as the persistent kernel's leaf body on a chain-row arena: one workgroup per
// chain, the potential's gradient read from g_eval instead of computed, the scalar state from
// and to the arena, the chain appended to the compacted list when its next leaf is pending.
// Replaces the four D-slice kernels (V1, R, S, V2), whose chain groups move at the pace of
// their slowest chain.  Same per-chain arithmetic as the persistent kernel.
struct RowsAll {
  int dim;
  static constexpr int NSCALAR = 0;
  NMX_HD int lo() const { return 0; }
  NMX_HD int hi() const { return dim; }
  NMX_HD int scalar_row(int) const { return 0; }
};

template <int NT, int B>
__global__ __launch_bounds__(NT, NMX_PX_OCC) void k_chain_step(StepArgs Pk) {
  constexpr int NW = NT / 64;
  __shared__ float lds[NPART * NW];
  __shared__ float lds_tot[NPART];
  __shared__ float lds_ke[NW];
  __shared__ int sh_act, sh_slot, sh_wfn, sh_it;
  __shared__ float sh_seff, sh_pe;
  const StepArgs& P = Pk;
  const nmx_nuts_config& cfg = P.cfg;
  const Arena& a = P.a;
  const int c = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // the list of the other parity was consumed by the last potential launch: clear it for the next step
  if (blockIdx.x == 0 && tid == 0) a.counters[2 + (cfg.parity ^ 1)] = 0;
  const int D = cfg.dim, ldc = cfg.ldc;
  const bool is_nuts = cfg.algo == NMX_ALGO_NUTS;
  const uint32_t gch = (uint32_t)(cfg.chain_offset + c);
  const uint64_t seed = cfg.seed;
  int ph = uni_i(AI(NMX_F_PHASE)[c]);  // the same for every wave: only this workgroup writes it
  if (ph == NMX_PH_DONE) return;
  if (ph == NMX_PH_WAIT) {  // sync_chains: start once every chain finished the transition
    // one thread reads the count for the whole workgroup (wait_released: waves reading it
    // separately could disagree while other workgroups are still adding to it)
    __shared__ int sh_go;
    if (tid == 0) sh_go = wait_released(cfg, a, AI(NMX_F_ITER)[c]) ? 1 : 0;
    __syncthreads();
    if (!uni_i(sh_go)) return;
    ph = NMX_PH_START;
  }
  Act A;
  {
    ChainScalars Sb;
    Sb.dir = uni_i(AI(NMX_F_DIR)[c]);
    Sb.sub_n = uni_i(AI(NMX_F_SUB_N)[c]);
    Sb.depth = uni_i(AI(NMX_F_DEPTH)[c]);
    begin_act(cfg, Sb, ph, A);
  }
  const VecCtx v{&a, ldc, D, (size_t)D * ldc, cfg.unit_mass != 0};
  const uint32_t base = ((uint32_t)c * (uint32_t)D) << 2;
  const RowsAll rows{D};
  if (A.leaf) {
    const float seff = uni_f(AF(NMX_F_STEP_EFF)[c]);
    const float* GE = AV(NMX_F_G_EVAL);
    {
      float red[NPART];
#pragma unroll
      for (int i = 0; i < NPART; ++i) red[i] = 0.0f;
      float dl = 0.0f, dr = 0.0f;
      for (int d0 = tid; d0 < D; d0 += B * NT) {
        PRow x[B];
        float g[B];
#pragma unroll
        for (int q = 0; q < B; ++q) {
          const int d = d0 + q * NT;
          if (d < D) {
            const uint32_t off = base + ((uint32_t)d << 2);
            g[q] = nmx_at(GE, off);
            if (is_nuts) prow_load<true>(v, A, off, x[q]);
            else prow_load<false>(v, A, off, x[q]);
          }
        }
#pragma unroll
        for (int q = 0; q < B; ++q) {
          const int d = d0 + q * NT;
          if (d < D) {
            const uint32_t off = base + ((uint32_t)d << 2);
            if (is_nuts) prow_store<true>(v, A, seff, off, x[q], g[q], red, dl, dr);
            else prow_store<false>(v, A, seff, off, x[q], g[q], red, dl, dr);
          }
        }
      }
      if (is_nuts) {
#pragma unroll
        for (int i = 0; i < MAXD; ++i)
          if (i == A.imin && A.imin <= A.imax) {
            red[1 + 2 * i] = dl;
            red[2 + 2 * i] = dr;
          }
      }
      wave_sums_to_lds<NW, NPART>(red, lds, A, is_nuts);
    }
    if (is_nuts && A.imax > A.imin) persist_ckpt_levels<NW, NT>(v, A, rows, base, lds);
    __syncthreads();
    if (wv == 0) {
      float tot = 0.0f;
      if (lane < NPART && entry_used(A, is_nuts, lane)) {
#pragma unroll
        for (int w = 0; w < NW; ++w) tot += lds[lane * NW + w];
      }
      if (lane < NPART) lds_tot[lane] = tot;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  // scalar logic: wave 0 (lane 0 writes the state back, the counters and the list entry)
  if (wv == 0) {
    ChainScalars S;
    load_scalars(a, c, S);
    A.pe_eval = A.leaf ? AF(NMX_F_PE_EVAL)[c] : 0.0f;
    leaf_phase(cfg, S, A, A.leaf ? 0.5f * lds_tot[0] : 0.0f, seed, gch);
    tree_phase(
        cfg, S, A, [&](int i, int side) { return lds_tot[1 + 2 * i + side]; },
        [&](int side) { return lds_tot[1 + 2 * MAXD + side]; }, seed, gch, P.fields, c, lane == 0);
    if (lane == 0) {
      store_scalars(a, c, S);
      sh_act = pack_act(A);
      sh_slot = A.slot;
      sh_wfn = A.wfn;
      sh_it = S.it;
      sh_seff = S.step_eff;
      sh_pe = S.pe;
      if (A.fin_done) atomicAdd(&a.counters[0], 1);
      if (A.fin_wait) {
        const int fs = A.fin_t - cfg.iter_begin;
        if (fs >= 0 && fs < cfg.iter_capacity) atomicAdd(&a.finished[fs], 1);
      }
      if (A.start_iter || A.prep_leaf) {  // the next leaf is pending: list it for the potential
        const int pos = atomicAdd(&a.counters[2 + cfg.parity], 1);
        NMX_DCHECK(pos < cfg.num_chains);
        a.active_idx[(size_t)cfg.parity * ldc + pos] = c;
      }
    }
  }
  __syncthreads();  // decisions published
  const int act = uni_i(sh_act);
  Act D2{};
  D2.take_leaf = act & ACT_TAKE_LEAF;
  D2.done_sub = act & ACT_DONE_SUB;
  D2.take_biased = act & ACT_TAKE_BIASED;
  D2.hmc_accept = act & ACT_HMC_ACCEPT;
  D2.iter_done = act & ACT_ITER_DONE;
  D2.wf_update = act & ACT_WF_UPDATE;
  D2.finalize = act & ACT_FINALIZE;
  D2.start_iter = act & ACT_START;
  D2.prep_leaf = act & ACT_PREP;
  D2.dirR = (act & ACT_DIRR) ? 1 : 0;
  D2.new_dir = (act & ACT_NEWDIR) ? 1 : 0;
  D2.slot = uni_i(sh_slot);
  D2.wfn = uni_i(sh_wfn);
  constexpr int VEC = ACT_TAKE_LEAF | ACT_DONE_SUB | ACT_TAKE_BIASED | ACT_HMC_ACCEPT | ACT_ITER_DONE | ACT_START |
                      ACT_PREP;
  float ke0 = 0.0f;
  constexpr int RARE = ACT_DONE_SUB | ACT_TAKE_BIASED | ACT_HMC_ACCEPT | ACT_ITER_DONE | ACT_WF_UPDATE |
                       ACT_FINALIZE | ACT_START;
  if (NMX_PX_FAST_APPLY && (act & ACT_PREP) && !(act & RARE) && D2.new_dir == D2.dirR) {
    apply_prep_rows_arena<NT, B>(v, D2, rows, uni_f(sh_seff), base);
  } else if (act & VEC) {
    float* const samp = (D2.iter_done && D2.slot >= 0 && P.samples) ? P.samples + (size_t)D2.slot * D * ldc : nullptr;
    ke0 = persist_apply_rows<NT, B>(v, D2, rows, uni_f(sh_seff), base, c, seed, gch, uni_i(sh_it), samp, P.transform,
                                    cfg);
  }
  if (D2.start_iter) {
    const float t = wave_sum(ke0);
    if (lane == 0) lds_ke[wv] = t;
    __syncthreads();
    if (tid == 0) {
      float tot = 0.0f;
#pragma unroll
      for (int w = 0; w < NW; ++w) tot += lds_ke[w];
      const float e0 = sh_pe + 0.5f * tot;  // build_tree :1130
      AF(NMX_F_E0)[c] = e0;
      AF(NMX_F_ENERGY)[c] = e0;  // proposal energy of the initial tree (:1137)
    }
  }
}
// ---------------------------------------------------------------------------------------
// Reset / init kernels (either arena layout: vidx)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ size_t vidx(const nmx_nuts_config& cfg, int d, int c) {
  return cfg.layout == NMX_LAYOUT_CHAIN_ROWS ? (size_t)c * cfg.dim + d : (size_t)d * cfg.ldc + c;
}

__global__ void k_nuts_reset(Arena a, nmx_nuts_config cfg, float step_size, const float* imm) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int ldc = cfg.ldc;
  if (c < ldc) {
    const bool valid = c < cfg.num_chains;
    for (int f = 0; f < NUM_INT_SCALARS; ++f) AI(NMX_F_PHASE + f)[c] = 0;
    for (int f = 0; f < NUM_FLOAT_SCALARS; ++f) AF(NMX_F_STEP_SIZE + f)[c] = 0.0f;
    AI(NMX_F_PHASE)[c] = valid ? NMX_PH_NEEDINIT : NMX_PH_DONE;
    AF(NMX_F_STEP_SIZE)[c] = step_size;
    AF(NMX_F_STEP_EFF)[c] = step_size;
    AF(NMX_F_DA_PROX)[c] = logf(10.0f * step_size);  // warmup_adapter init_fn :576
    for (int d = 0; d < cfg.dim; ++d) {
      const size_t idx = vidx(cfg, d, c);
      const float im = imm ? imm[d] : 1.0f;
      AV(NMX_F_INV_MASS)[idx] = im;
      // _initialize_mass_matrix diag branch (:507-512): sqrt_inv = sqrt(imm), sqrt = 1/that
      AV(NMX_F_MASS_SQRT)[idx] = imm ? 1.0f / sqrtf(im) : 1.0f;
      AV(NMX_F_WF_MEAN)[idx] = 0.0f;
      AV(NMX_F_WF_M2)[idx] = 0.0f;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < 16) a.counters[threadIdx.x] = 0;
  for (int i = c; i < cfg.iter_capacity; i += gridDim.x * blockDim.x) a.finished[i] = 0;
}

__global__ void k_nuts_init_draw(Arena a, nmx_nuts_config cfg, int attempt, float radius) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cfg.num_chains) return;
  if (AI(NMX_F_PHASE)[c] != NMX_PH_NEEDINIT) return;
  const uint32_t gch = (uint32_t)(cfg.chain_offset + c);
  for (int blk = 0; 4 * blk < cfg.dim; ++blk) {
    const nmx_u4 x = nmx_rng(cfg.seed, gch, 0, NMX_EV_INIT, blk, (uint32_t)attempt);
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int d = 4 * blk + q;
      if (d < cfg.dim) AV(NMX_F_Z_EVAL)[vidx(cfg, d, c)] = (2.0f * radius) * nmx_u01(w[q]) - radius;
    }
  }
  AI(NMX_F_PHASE)[c] = NMX_PH_INITEVAL;
}

__global__ void k_nuts_init_from(Arena a, nmx_nuts_config cfg, const float* z) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cfg.num_chains) return;
  const int ldc = cfg.ldc;  // z is [D][ldc] in either arena layout
  for (int d = 0; d < cfg.dim; ++d) AV(NMX_F_Z_EVAL)[vidx(cfg, d, c)] = z[(size_t)d * ldc + c];
  AI(NMX_F_PHASE)[c] = NMX_PH_INITEVAL;
}

__global__ void k_nuts_init_check(Arena a, nmx_nuts_config cfg) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cfg.num_chains) return;
  const int ph = AI(NMX_F_PHASE)[c];
  if (ph == NMX_PH_INITEVAL) {
    const float pe = AF(NMX_F_PE_EVAL)[c];
    bool ok = isfinite(pe);
    for (int d = 0; d < cfg.dim; ++d) ok = ok && isfinite(AV(NMX_F_G_EVAL)[vidx(cfg, d, c)]);
    if (ok) {
      for (int d = 0; d < cfg.dim; ++d) {
        const size_t idx = vidx(cfg, d, c);
        AV(NMX_F_Z)[idx] = AV(NMX_F_Z_EVAL)[idx];
        AV(NMX_F_ZGRAD)[idx] = AV(NMX_F_G_EVAL)[idx];
      }
      AF(NMX_F_PE)[c] = pe;
      AF(NMX_F_ENERGY)[c] = pe;
      AI(NMX_F_PHASE)[c] = NMX_PH_START;
    } else {
      AI(NMX_F_PHASE)[c] = NMX_PH_NEEDINIT;
      atomicAdd(&a.counters[1], 1);
    }
  } else if (ph == NMX_PH_NEEDINIT) {
    atomicAdd(&a.counters[1], 1);
  }
}

__global__ void k_nuts_resume(Arena a, nmx_nuts_config cfg) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < 16) a.counters[threadIdx.x] = 0;
  for (int i = c; i < cfg.iter_capacity; i += gridDim.x * blockDim.x) a.finished[i] = 0;
  if (c >= cfg.num_chains) return;
  const int ph = AI(NMX_F_PHASE)[c];
  if (ph == NMX_PH_DONE || ph == NMX_PH_WAIT || ph == NMX_PH_START) AI(NMX_F_PHASE)[c] = NMX_PH_START;
}

// ---- find_reasonable_step_size (hmc_util.py:314-384) ----------------------------------
// Per chain, from its stored state (z, U, grad): repeat { step *= 2^direction; r = momentum;
// one velocity_verlet step; direction' = log(0.8) < -dE ? 1 : -1 } while the direction keeps
// its sign and the step stays within (tiny, max).  The reference draws the momentum as
// momentum_generator(z, inverse_mass_matrix, key) (hmc_util.py:359), i.e. r = M^-1 eps (the
// inverse mass where momentum_generator expects its square root); reproduced as is.
// HS_K = attempt count (-1: search finished), HS_DIR / HS_LAST = direction / last direction,
// HS_STEP = step, HS_E0 = energy of the attempt's start; RL holds r(n+1/2) of the attempt.
__global__ void k_heur_begin(Arena a, nmx_nuts_config cfg) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.counters[1] = 0;
  if (c >= cfg.num_chains) return;
  AI(NMX_F_HS_K)[c] = 0;
  AI(NMX_F_HS_DIR)[c] = 0;
  AI(NMX_F_HS_LAST)[c] = 0;
  AF(NMX_F_HS_STEP)[c] = AF(NMX_F_STEP_SIZE)[c];
}

// the search's normals of every searching chain's attempt, eps[D][ldc] (0 for the others):
// the momentum draw of k_heur_propose, exported for a caller that maps it through a dense mass
__global__ void k_heur_noise(Arena a, nmx_nuts_config cfg, float* eps) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cfg.ldc) return;
  const int k = c < cfg.num_chains ? AI(NMX_F_HS_K)[c] : -1;
  const uint32_t gch = (uint32_t)(cfg.chain_offset + c);
  const int it = k >= 0 ? AI(NMX_F_ITER)[c] : 0;
  for (int blk = 0; 4 * blk < cfg.dim; ++blk) {
    float n[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (k >= 0) {
      const nmx_u4 x = nmx_rng(cfg.seed, gch, (uint32_t)it, NMX_EV_HEURISTIC, blk, (uint32_t)k);
      nmx_box_muller(x.x, x.y, n[0], n[1]);
      nmx_box_muller(x.z, x.w, n[2], n[3]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * blk + q < cfg.dim) eps[(size_t)(4 * blk + q) * cfg.ldc + c] = n[q];
  }
}

// step update, momentum, first half step and z_eval; lists the searching chains (list 0).
// mom != NULL: the momentum is given ([D][ldc], unit mass: a whitened dense mass's
// T^T M^-1 eps), else drawn as im * eps (hmc_util.py:359 momentum_generator)
__global__ void k_heur_propose(Arena a, nmx_nuts_config cfg, const float* mom) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = c < cfg.num_chains ? AI(NMX_F_HS_K)[c] : -1;
  const bool act = k >= 0;
  if (act) {
    const int dir = AI(NMX_F_HS_DIR)[c];
    const float step = AF(NMX_F_HS_STEP)[c] * (dir > 0 ? 2.0f : (dir < 0 ? 0.5f : 1.0f));
    AF(NMX_F_HS_STEP)[c] = step;
    const uint32_t gch = (uint32_t)(cfg.chain_offset + c);
    const int it = AI(NMX_F_ITER)[c];
    const int ldc = cfg.ldc;
    float ke = 0.0f;
    for (int blk = 0; 4 * blk < cfg.dim; ++blk) {
      float n[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (!mom) {
        const nmx_u4 x = nmx_rng(cfg.seed, gch, (uint32_t)it, NMX_EV_HEURISTIC, blk, (uint32_t)k);
        nmx_box_muller(x.x, x.y, n[0], n[1]);
        nmx_box_muller(x.z, x.w, n[2], n[3]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = 4 * blk + q;
        if (d < cfg.dim) {
          const size_t idx = (size_t)d * ldc + c;
          const float im = cfg.unit_mass ? 1.0f : AV(NMX_F_INV_MASS)[idx];
          const float r = mom ? mom[idx] : im * n[q];
          ke += (im * r) * r;
          const float rh = r - (0.5f * step) * AV(NMX_F_ZGRAD)[idx];
          AV(NMX_F_RL)[idx] = rh;
          AV(NMX_F_Z_EVAL)[idx] = AV(NMX_F_Z)[idx] + step * (im * rh);
        }
      }
    }
    AF(NMX_F_HS_E0)[c] = 0.5f * ke + AF(NMX_F_PE)[c];  // kinetic_fn(imm, r) + potential_energy
  }
  const int lane = threadIdx.x & 63;
  const uint64_t m = __ballot(act);
  if (m) {
    int base = 0;
    if (lane == __builtin_ctzll(m)) base = atomicAdd(&a.counters[2], __builtin_popcountll(m));
    base = __shfl(base, __builtin_ctzll(m));
    if (act) a.active_idx[base + __builtin_popcountll(m & ((1ull << lane) - 1ull))] = c;
  }
}

// second half step, energy change, new direction; a chain whose search ends stores its step
// size and restarts dual averaging at it (warmup_adapter :573-576 at init, :619-626 at window
// ends); counters[1] = chains still searching
__global__ void k_heur_finish(Arena a, nmx_nuts_config cfg, int at_init) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.counters[2]) return;
  const int c = a.active_idx[p];
  const int ldc = cfg.ldc;
  const float step = AF(NMX_F_HS_STEP)[c];
  float ke = 0.0f;
  for (int d = 0; d < cfg.dim; ++d) {
    const size_t idx = (size_t)d * ldc + c;
    const float im = cfg.unit_mass ? 1.0f : AV(NMX_F_INV_MASS)[idx];
    const float r = AV(NMX_F_RL)[idx] - (0.5f * step) * AV(NMX_F_G_EVAL)[idx];
    ke += (im * r) * r;
  }
  const float dE = (0.5f * ke + AF(NMX_F_PE_EVAL)[c]) - AF(NMX_F_HS_E0)[c];
  const int dir_new = logf(0.8f) < -dE ? 1 : -1;  // NaN dE -> -1
  const int last = AI(NMX_F_HS_DIR)[c];
  AI(NMX_F_HS_LAST)[c] = last;
  AI(NMX_F_HS_DIR)[c] = dir_new;
  const bool not_small = step > 1.17549435e-38f || dir_new >= 0;
  const bool not_large = step < 3.40282347e+38f || dir_new <= 0;
  if (not_small && not_large && (last == 0 || dir_new == last)) {
    AI(NMX_F_HS_K)[c] = AI(NMX_F_HS_K)[c] + 1;
    atomicAdd(&a.counters[1], 1);
  } else {
    AI(NMX_F_HS_K)[c] = -1;
    AF(NMX_F_STEP_SIZE)[c] = step;
    AF(NMX_F_STEP_EFF)[c] = step;
    AF(NMX_F_DA_PROX)[c] = at_init ? logf(10.0f * step) : logf(10.0f) + logf(step);
    AF(NMX_F_DA_XT)[c] = 0.0f;
    AF(NMX_F_DA_XAVG)[c] = 0.0f;
    AF(NMX_F_DA_GAVG)[c] = 0.0f;
    AI(NMX_F_DA_T)[c] = 0;
  }
}

int validate(const nmx_nuts_config* cfg) {
  if (!cfg) return nmx_fail(NMX_ERR_INVALID, "config is NULL");
  if (cfg->num_chains <= 0 || cfg->dim <= 0) return nmx_fail(NMX_ERR_INVALID, "num_chains and dim must be positive");
  if (cfg->algo != NMX_ALGO_NUTS && cfg->algo != NMX_ALGO_HMC)
    return nmx_fail(NMX_ERR_INVALID, "algo must be NUTS(0) or HMC(1)");
  if (cfg->unit_mass && cfg->adapt_mass_matrix)
    return nmx_fail(NMX_ERR_INVALID, "unit_mass excludes adapt_mass_matrix");
  const int md = cfg->max_tree_depth > cfg->max_tree_depth_warmup ? cfg->max_tree_depth : cfg->max_tree_depth_warmup;
  if (cfg->algo == NMX_ALGO_NUTS) {
    if (cfg->max_tree_depth < 1 || cfg->max_tree_depth_warmup < 1)
      return nmx_fail(NMX_ERR_INVALID, "max_tree_depth must be >= 1");
    if (md > NMX_MAX_TREE_DEPTH || md > cfg->max_depth_alloc)
      return nmx_fail(NMX_ERR_INVALID, "max_tree_depth %d exceeds allocation (%d, limit %d)", md,
                      cfg->max_depth_alloc, NMX_MAX_TREE_DEPTH);
  }
  if (cfg->num_windows < 1 || cfg->num_windows > NMX_MAX_WINDOWS)
    return nmx_fail(NMX_ERR_INVALID, "num_windows out of range");
  if (cfg->collect_thinning < 1) return nmx_fail(NMX_ERR_INVALID, "collect_thinning must be >= 1");
  if (cfg->sync_chains && cfg->iter_capacity < cfg->iter_end - cfg->iter_begin)
    return nmx_fail(NMX_ERR_INVALID, "sync_chains needs iter_capacity >= iter_end - iter_begin");
  if (cfg->algo == NMX_ALGO_HMC && cfg->num_steps <= 0 && !(cfg->trajectory_length > 0.0f))
    return nmx_fail(NMX_ERR_INVALID, "HMC needs num_steps or trajectory_length");
  if (cfg->ldc != ldc_of(cfg->num_chains))
    return nmx_fail(NMX_ERR_INVALID, "cfg.ldc must be round_up(num_chains, 64) = %d", ldc_of(cfg->num_chains));
  if (cfg->layout != NMX_LAYOUT_CHAIN_MINOR && cfg->layout != NMX_LAYOUT_CHAIN_ROWS)
    return nmx_fail(NMX_ERR_INVALID, "layout must be NMX_LAYOUT_CHAIN_MINOR(0) or NMX_LAYOUT_CHAIN_ROWS(1)");
  if (cfg->num_groups < 0 || cfg->num_groups == 3 || cfg->num_groups > 4)
    return nmx_fail(NMX_ERR_INVALID, "num_groups must be 0, 1, 2 or 4");
  if (cfg->group < 0 || cfg->group >= group_count(*cfg)) return nmx_fail(NMX_ERR_INVALID, "group out of range");
  return NMX_OK;
}

// the launched schedules index vectors [D][ldc]
int need_chain_minor(const nmx_nuts_config* cfg, const char* what) {
  if (cfg->layout != NMX_LAYOUT_CHAIN_MINOR)
    return nmx_fail(NMX_ERR_INVALID, "%s needs the chain-minor arena layout (NMX_LAYOUT_CHAIN_MINOR)", what);
  return NMX_OK;
}

Arena arena_of(const nmx_nuts_config* cfg, void* base) {
  return make_arena(base, cfg->ldc, cfg->dim, cfg->max_depth_alloc, cfg->iter_capacity);
}

// fused schedule only (D < WIDE_MIN_D)
int tpc_for_dim(int D) { return D < 16 ? 1 : 8; }

}  // namespace

extern "C" int nmx_nuts_num_slices(int dim) { return num_slices(dim); }

extern "C" size_t nmx_nuts_arena_bytes(int num_chains, int dim, int max_depth_alloc, int iter_capacity) {
  const int ldc = ldc_of(num_chains);
  return field_offset(NMX_NUM_FIELDS, ldc, dim, max_depth_alloc, iter_capacity);
}

extern "C" int nmx_nuts_field_info(int num_chains, int dim, int max_depth_alloc, int iter_capacity,
                                   int field, size_t* offset, size_t* nbytes) {
  if (field < 0 || field >= NMX_NUM_FIELDS) return nmx_fail(NMX_ERR_INVALID, "bad field %d", field);
  const int ldc = ldc_of(num_chains);
  if (offset) *offset = field_offset(field, ldc, dim, max_depth_alloc, iter_capacity);
  if (nbytes) *nbytes = field_bytes(field, ldc, dim, max_depth_alloc, iter_capacity);
  return NMX_OK;
}

extern "C" int nmx_nuts_reset(const nmx_nuts_config* cfg, void* arena, float step_size,
                              const float* inverse_mass_diag, void* stream) {
  int st = validate(cfg);
  if (st) return st;
  if (!arena) return nmx_fail(NMX_ERR_INVALID, "arena is NULL");
  Arena a = arena_of(cfg, arena);
  const int grid = (cfg->ldc + 63) / 64;
  hipLaunchKernelGGL(k_nuts_reset, dim3(grid), dim3(64), 0, (hipStream_t)stream, a, *cfg,
                     step_size, inverse_mass_diag);
  return nmx_check_launch("k_nuts_reset");
}

extern "C" int nmx_nuts_init_draw(const nmx_nuts_config* cfg, void* arena, int attempt, float radius,
                                  void* stream) {
  int st = validate(cfg);
  if (st) return st;
  Arena a = arena_of(cfg, arena);
  hipLaunchKernelGGL(k_nuts_init_draw, dim3((cfg->num_chains + 63) / 64), dim3(64), 0,
                     (hipStream_t)stream, a, *cfg, attempt, radius);
  return nmx_check_launch("k_nuts_init_draw");
}

extern "C" int nmx_nuts_init_from(const nmx_nuts_config* cfg, void* arena, const float* z, void* stream) {
  int st = validate(cfg);
  if (st) return st;
  if (!z) return nmx_fail(NMX_ERR_INVALID, "z is NULL");
  Arena a = arena_of(cfg, arena);
  hipLaunchKernelGGL(k_nuts_init_from, dim3((cfg->num_chains + 63) / 64), dim3(64), 0,
                     (hipStream_t)stream, a, *cfg, z);
  return nmx_check_launch("k_nuts_init_from");
}

extern "C" int nmx_nuts_init_check(const nmx_nuts_config* cfg, void* arena, void* stream) {
  int st = validate(cfg);
  if (st) return st;
  Arena a = arena_of(cfg, arena);
  if (hipMemsetAsync(a.counters + 1, 0, 4, (hipStream_t)stream) != hipSuccess)
    return nmx_fail(NMX_ERR_HIP, "hipMemsetAsync failed");
  hipLaunchKernelGGL(k_nuts_init_check, dim3((cfg->num_chains + 63) / 64), dim3(64), 0,
                     (hipStream_t)stream, a, *cfg);
  return nmx_check_launch("k_nuts_init_check");
}

extern "C" int nmx_heuristic_begin(const nmx_nuts_config* cfg, void* arena, void* stream) {
  int st = validate(cfg);
  if (st) return st;
  if ((st = need_chain_minor(cfg, "nmx_heuristic_begin"))) return st;
  if (group_count(*cfg) > 1) return nmx_fail(NMX_ERR_INVALID, "nmx_heuristic_begin: one chain group only");
  Arena a = arena_of(cfg, arena);
  hipLaunchKernelGGL(k_heur_begin, dim3((cfg->num_chains + 63) / 64), dim3(64), 0, (hipStream_t)stream, a, *cfg);
  return nmx_check_launch("k_heur_begin");
}

extern "C" int nmx_heuristic_propose_with(const nmx_nuts_config* cfg, void* arena, const float* momentum,
                                          void* stream) {
  int st = validate(cfg);
  if (st) return st;
  if ((st = need_chain_minor(cfg, "nmx_heuristic_propose"))) return st;
  if (group_count(*cfg) > 1) return nmx_fail(NMX_ERR_INVALID, "nmx_heuristic_propose: one chain group only");
  if (momentum && !cfg->unit_mass)
    return nmx_fail(NMX_ERR_INVALID, "nmx_heuristic_propose_with: a given momentum needs unit_mass");
  Arena a = arena_of(cfg, arena);
  if (hipMemsetAsync(a.counters + 2, 0, 4, (hipStream_t)stream) != hipSuccess)
    return nmx_fail(NMX_ERR_HIP, "hipMemsetAsync failed");
  hipLaunchKernelGGL(k_heur_propose, dim3((cfg->num_chains + 63) / 64), dim3(64), 0, (hipStream_t)stream, a,
                     *cfg, momentum);
  return nmx_check_launch("k_heur_propose");
}

extern "C" int nmx_heuristic_propose(const nmx_nuts_config* cfg, void* arena, void* stream) {
  return nmx_heuristic_propose_with(cfg, arena, nullptr, stream);
}

extern "C" int nmx_heuristic_noise(const nmx_nuts_config* cfg, void* arena, float* eps, void* stream) {
  int st = validate(cfg);
  if (st) return st;
  if ((st = need_chain_minor(cfg, "nmx_heuristic_noise"))) return st;
  if (!eps) return nmx_fail(NMX_ERR_INVALID, "nmx_heuristic_noise: eps is NULL");
  Arena a = arena_of(cfg, arena);
  hipLaunchKernelGGL(k_heur_noise, dim3(cfg->ldc / 64), dim3(64), 0, (hipStream_t)stream, a, *cfg, eps);
  return nmx_check_launch("k_heur_noise");
}

extern "C" int nmx_heuristic_finish(const nmx_nuts_config* cfg, void* arena, int at_init, void* stream) {
  int st = validate(cfg);
  if (st) return st;
  if ((st = need_chain_minor(cfg, "nmx_heuristic_finish"))) return st;
  if (group_count(*cfg) > 1) return nmx_fail(NMX_ERR_INVALID, "nmx_heuristic_finish: one chain group only");
  Arena a = arena_of(cfg, arena);
  if (hipMemsetAsync(a.counters + 1, 0, 4, (hipStream_t)stream) != hipSuccess)
    return nmx_fail(NMX_ERR_HIP, "hipMemsetAsync failed");
  hipLaunchKernelGGL(k_heur_finish, dim3((cfg->num_chains + 63) / 64), dim3(64), 0, (hipStream_t)stream, a,
                     *cfg, at_init);
  return nmx_check_launch("k_heur_finish");
}

extern "C" int nmx_nuts_resume(const nmx_nuts_config* cfg, void* arena, void* stream) {
  int st = validate(cfg);
  if (st) return st;
  Arena a = arena_of(cfg, arena);
  hipLaunchKernelGGL(k_nuts_resume, dim3((cfg->ldc + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     a, *cfg);
  return nmx_check_launch("k_nuts_resume");
}

extern "C" int nmx_nuts_run_small(const nmx_nuts_config* cfg, void* arena, float* samples, float* fields,
                                  const int8_t* transform, int model, const float* p0, const float* p1, int n,
                                  int max_steps, void* stream) {
  int st = validate(cfg);
  if (st) return st;
  if ((st = need_chain_minor(cfg, "nmx_nuts_run_small"))) return st;
  if (group_count(*cfg) > 1) return nmx_fail(NMX_ERR_INVALID, "nmx_nuts_run_small: one chain group only");
  if (!arena) return nmx_fail(NMX_ERR_INVALID, "arena is NULL");
  // samples may be NULL: the per-transition fields alone are collected
  if (cfg->collection_size > 0 && (!fields || !transform))
    return nmx_fail(NMX_ERR_INVALID, "collection buffers are NULL");
  if (tpc_for_dim(cfg->dim) != 1 || num_slices(cfg->dim) != 0)
    return nmx_fail(NMX_ERR_INVALID, "run_small: dim %d is not a one-wave model (dim < 16)", cfg->dim);
  if (cfg->sync_chains) return nmx_fail(NMX_ERR_INVALID, "run_small: the persistent schedule is per-chain async");
  if (!p0 || !p1 || max_steps <= 0) return nmx_fail(NMX_ERR_INVALID, "run_small: bad model parameters");
  StepArgs args;
  args.a = arena_of(cfg, arena);
  args.cfg = *cfg;
  args.samples = samples;
  args.fields = fields;
  args.transform = transform;
  const dim3 grid((cfg->num_chains + SMALL_CPW - 1) / SMALL_CPW), blk(64);
  hipStream_t s = (hipStream_t)stream;
  if (model == NMX_SMALL_DIAG_NORMAL) {
    if (n != cfg->dim) return nmx_fail(NMX_ERR_INVALID, "run_small: diag_normal needs n == dim");
    hipLaunchKernelGGL(k_nuts_persistent<NmxDiagNormal>, grid, blk, 0, s, args, NmxDiagNormal{p0, p1, n}, max_steps);
  } else if (model == NMX_SMALL_EIGHT_SCHOOLS) {
    if (n + 2 != cfg->dim) return nmx_fail(NMX_ERR_INVALID, "run_small: eight_schools needs dim == J + 2");
    hipLaunchKernelGGL(k_nuts_persistent<NmxEightSchools>, grid, blk, 0, s, args, NmxEightSchools{p0, p1, n},
                       max_steps);
  } else {
    return nmx_fail(NMX_ERR_INVALID, "run_small: unknown model %d", model);
  }
  return nmx_check_launch("k_nuts_persistent");
}

namespace {
int persist_nt(int dim);
// nmx_nuts_step on a chain-row arena: the per-chain step kernel (D-split dims only)
int step_chain_rows(const nmx_nuts_config* cfg, void* arena, float* samples, float* fields, const int8_t* transform,
                    void* stream) {
  if (num_slices(cfg->dim) == 0)
    return nmx_fail(NMX_ERR_INVALID, "step: the chain-row layout is for dim >= %d", WIDE_MIN_D);
  if (group_count(*cfg) > 1) return nmx_fail(NMX_ERR_INVALID, "step: chain-row layout, one chain group only");
  if (cfg->parity != 0 && cfg->parity != 1) return nmx_fail(NMX_ERR_INVALID, "parity must be 0 or 1");
  if (cfg->collection_size > 0 && (!fields || !transform))
    return nmx_fail(NMX_ERR_INVALID, "collection buffers are NULL");
  if ((size_t)cfg->ldc * cfg->dim * 4 > 0xFFFFFFF0ull)
    return nmx_fail(NMX_ERR_INVALID, "step: a vector field exceeds 4 GiB");
  StepArgs args;
  args.a = arena_of(cfg, arena);
  args.cfg = *cfg;
  args.samples = samples;
  args.fields = fields;
  args.transform = transform;
  const dim3 grid(cfg->num_chains);
  hipStream_t s = (hipStream_t)stream;
  switch (persist_nt(cfg->dim)) {
    case 128: hipLaunchKernelGGL((k_chain_step<128, NMX_PX_B>), grid, dim3(128), 0, s, args); break;
    case 256: hipLaunchKernelGGL((k_chain_step<256, NMX_PX_B>), grid, dim3(256), 0, s, args); break;
    case 512: hipLaunchKernelGGL((k_chain_step<512, NMX_PX_B>), grid, dim3(512), 0, s, args); break;
    default: hipLaunchKernelGGL((k_chain_step<1024, NMX_PX_B>), grid, dim3(1024), 0, s, args);
  }
  return nmx_check_launch("k_chain_step");
}
}  // namespace

extern "C" int nmx_nuts_step(const nmx_nuts_config* cfg, void* arena, float* samples, float* fields,
                             const int8_t* transform, void* stream) {
  int st = validate(cfg);
  if (st) return st;
  if (!arena) return nmx_fail(NMX_ERR_INVALID, "arena is NULL");
  if (cfg->layout == NMX_LAYOUT_CHAIN_ROWS) return step_chain_rows(cfg, arena, samples, fields, transform, stream);
  // samples may be NULL: the per-transition fields alone are collected
  if (cfg->collection_size > 0 && (!fields || !transform))
    return nmx_fail(NMX_ERR_INVALID, "collection buffers are NULL");
  StepArgs args;
  args.a = arena_of(cfg, arena);
  args.cfg = *cfg;
  args.samples = samples;
  args.fields = fields;
  args.transform = transform;
  const int grid = cfg->ldc / 64;
  hipStream_t s = (hipStream_t)stream;
  if (cfg->parity != 0 && cfg->parity != 1) return nmx_fail(NMX_ERR_INVALID, "parity must be 0 or 1");
  const int ns = num_slices(cfg->dim);
  if (ns > 0 && group_count(*cfg) > 1)
    return nmx_fail(NMX_ERR_INVALID, "chain groups: the fused step only (dim <= 256)");
  if (ns > 0) {
    WideArgs w{args, ns, slice_width(cfg->dim)};
    hipLaunchKernelGGL(k_wide_v1, dim3(grid, ns), dim3(64 * WIDE_WAVES), 0, s, w);
    hipLaunchKernelGGL(k_wide_r, dim3(grid, NPART + 1), dim3(64 * WIDE_SWAVES), 0, s, w);
    hipLaunchKernelGGL(k_wide_s, dim3(grid), dim3(64), 0, s, w);
    hipLaunchKernelGGL(k_wide_v2, dim3(grid, ns), dim3(64 * V2_WAVES), 0, s, w);
    return nmx_check_launch("k_nuts_step (wide)");
  }
  // the blocks cover the launch's chain group (all chains with one group)
  const int gchains = group_count(*cfg) > 1 ? group_size(*cfg) : cfg->ldc;
  if (tpc_for_dim(cfg->dim) == 1)
    hipLaunchKernelGGL((k_nuts_step<1, SMALL_CPW>), dim3((gchains + SMALL_CPW - 1) / SMALL_CPW), dim3(64), 0, s, args);
  else
    hipLaunchKernelGGL((k_nuts_step<8, STEP_CPW>), dim3((gchains + STEP_CPW - 1) / STEP_CPW), dim3(512), 0, s, args);
  return nmx_check_launch("k_nuts_step");
}

extern "C" size_t nmx_nuts_wide_model_workspace_bytes(int dim, int num_chains) {
  const int ldc = ldc_of(num_chains);
  if (num_slices(dim) == 0) return 0;
  return wide_ws_part_bytes(dim, ldc) + wide_ws_tot_bytes(ldc) + align_up((size_t)(ldc / 64) * 4);
}

namespace {
template <class M>
int launch_wide_model(const WideArgs& w, const M& m, char* ws, int ldc, hipStream_t s) {
  float* ppart = (float*)ws;
  float* ptot = (float*)(ws + wide_ws_part_bytes(w.p.cfg.dim, ldc));
  int* cnt = (int*)(ws + wide_ws_part_bytes(w.p.cfg.dim, ldc) + wide_ws_tot_bytes(ldc));
  const int grid = ldc / 64;
  hipLaunchKernelGGL(k_wide_leaf<M>, dim3(grid, w.ns), dim3(64 * WIDE_WAVES), 0, s, w, m, ppart);
  hipLaunchKernelGGL(k_wide_rs<M>, dim3(grid, NPART + 1 + M::NSUM), dim3(64 * WIDE_SWAVES), 0, s, w, m,
                     (const float*)ppart, ptot, cnt);
  hipLaunchKernelGGL(k_wide_v2, dim3(grid, w.ns), dim3(64 * V2_WAVES), 0, s, w);
  return nmx_check_launch("nmx_nuts_step_wide_model");
}
}  // namespace

extern "C" int nmx_nuts_step_wide_model(const nmx_nuts_config* cfg, void* arena, float* samples, float* fields,
                                        const int8_t* transform, int model, const float* data, int n,
                                        void* workspace, void* stream) {
  int st = validate(cfg);
  if (st) return st;
  if ((st = need_chain_minor(cfg, "nmx_nuts_step_wide_model"))) return st;
  if (group_count(*cfg) > 1) return nmx_fail(NMX_ERR_INVALID, "nmx_nuts_step_wide_model: one chain group only");
  if (!arena || !workspace) return nmx_fail(NMX_ERR_INVALID, "arena / workspace is NULL");
  // samples may be NULL: the per-transition fields alone are collected
  if (cfg->collection_size > 0 && (!fields || !transform))
    return nmx_fail(NMX_ERR_INVALID, "collection buffers are NULL");
  const int ns = num_slices(cfg->dim);
  if (ns == 0) return nmx_fail(NMX_ERR_INVALID, "step_wide_model: dim %d uses the fused step (dim < %d)", cfg->dim,
                               WIDE_MIN_D);
  StepArgs args;
  args.a = arena_of(cfg, arena);
  args.cfg = *cfg;
  args.samples = samples;
  args.fields = fields;
  args.transform = transform;
  const WideArgs w{args, ns, slice_width(cfg->dim)};
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  switch (model) {
    case NMX_WIDE_STOCHASTIC_VOLATILITY:
      if (!data || n <= 1 || n + 2 != cfg->dim)
        return nmx_fail(NMX_ERR_INVALID, "step_wide_model: stochastic volatility needs returns[T], dim == T + 2");
      return launch_wide_model(w, NmxWideSV{data, n}, ws, cfg->ldc, s);
    case NMX_WIDE_FUNNEL:
      if (n != cfg->dim) return nmx_fail(NMX_ERR_INVALID, "step_wide_model: funnel needs n == dim");
      return launch_wide_model(w, NmxWideFunnel{n}, ws, cfg->ldc, s);
    case NMX_WIDE_FUNNEL_NONCENTERED:
      if (n != cfg->dim) return nmx_fail(NMX_ERR_INVALID, "step_wide_model: funnel_noncentered needs n == dim");
      return launch_wide_model(w, NmxWideFunnelNC{n}, ws, cfg->ldc, s);
    default:
      return nmx_fail(NMX_ERR_INVALID, "step_wide_model: unknown model %d", model);
  }
}

namespace {
// threads per chain of the persistent wide kernel, from dim only (the sums' order depends on
// it).  The NMX_PERSIST_NT environment override for kernel experiments exists only in the debug
// build and in experiment builds (-DNMX_EXPERIMENT, scripts/ab_build.py): the release library's
// results never depend on the environment.
int persist_nt(int dim) {
#if defined(NMX_DEBUG) || defined(NMX_EXPERIMENT)
  if (const char* e = getenv("NMX_PERSIST_NT")) {
    const int v = atoi(e);
    if (v == 128 || v == 256 || v == 512 || v == 1024) return v;
  }
#endif
  // SV (D = 2519): 256 -> 13.1M leapfrog/s at 8192 chains, 512 -> 9.6M; funnel-10k: 512 -> 5.1M,
  // 256 -> 4.7M (profiles/r03/ab_persistent_nt.txt)
  return dim <= 4096 ? 256 : 512;
}

// Whether the persistent kernel keeps the chain's frontier and inverse mass in LDS
// (k_wide_persistent CARRY): its 16 D bytes beside the static LDS must fit the share of a CU's
// 160 KB that the compiled occupancy (NMX_PX_OCC waves per SIMD, NT / 64 waves per workgroup)
// leaves each workgroup, so the carry never costs resident chains (SV D = 2519 at NT = 256:
// 40.9 KB of 40 KB; funnel-10k at NT = 512: 160 KB of 80, not carried).  No effect on results
// (bitwise equal either way); the debug / experiment builds can turn it off
// (NMX_PERSIST_CARRY=0) for A/B runs.
bool persist_carry(int dim, int nt, size_t static_lds) {
#if defined(NMX_DEBUG) || defined(NMX_EXPERIMENT)
  if (const char* e = getenv("NMX_PERSIST_CARRY"))
    if (atoi(e) == 0) return false;
#endif
  const size_t share = (size_t)160 * 1024 * nt / (64 * 4 * NMX_PX_OCC);
  return (size_t)16 * dim + static_lds <= share;
}

template <int NT, class M>
int launch_persistent_nt(const StepArgs& args, const M& m, int max_steps, hipStream_t s) {
  const dim3 grid(args.cfg.num_chains);
  if (persist_carry(args.cfg.dim, NT, (sizeof(PersistShared<NT, M, true>) + 15) / 16 * 16)) {
    const size_t lds = (size_t)16 * args.cfg.dim;
    if (const int st = nmx_lds_limit((const void*)k_wide_persistent<NT, NMX_PX_BA, M, true>, lds, s, "run_wide"))
      return st;
    hipLaunchKernelGGL((k_wide_persistent<NT, NMX_PX_BA, M, true>), grid, dim3(NT), lds, s, args, m, max_steps);
  } else {
    hipLaunchKernelGGL((k_wide_persistent<NT, NMX_PX_BA, M, false>), grid, dim3(NT), 0, s, args, m, max_steps);
  }
  return NMX_OK;
}

template <class M>
int launch_persistent(const StepArgs& args, const M& m, int max_steps, hipStream_t s) {
  int st;
  switch (persist_nt(args.cfg.dim)) {
    case 128: st = launch_persistent_nt<128>(args, m, max_steps, s); break;
    case 256: st = launch_persistent_nt<256>(args, m, max_steps, s); break;
    case 512: st = launch_persistent_nt<512>(args, m, max_steps, s); break;
    default: st = launch_persistent_nt<1024>(args, m, max_steps, s);
  }
  if (st != NMX_OK) return st;
  return nmx_check_launch("k_wide_persistent");
}
}  // namespace

#if defined(NMX_DEBUG) || defined(NMX_EXPERIMENT)
// kernel experiments: resident workgroups per CU of the persistent SV kernel at dim (and whether
// it carries the frontier in LDS), from the HIP occupancy calculator
extern "C" int nmx_debug_persist_occupancy(int dim, int* blocks_per_cu, int* carry) {
  const NmxWideSV m{nullptr, dim - 2};
  (void)m;
  const int nt = persist_nt(dim);
  if (nt != 256) return nmx_fail(NMX_ERR_UNSUPPORTED, "occupancy probe: NT = 256 dims only");
  const bool cr = persist_carry(dim, 256, (sizeof(PersistShared<256, NmxWideSV, true>) + 15) / 16 * 16);
  *carry = cr;
  hipError_t e;
  if (cr)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_wide_persistent<256, NMX_PX_BA, NmxWideSV, true>,
                                                     256, (size_t)16 * dim);
  else
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_wide_persistent<256, NMX_PX_BA, NmxWideSV, false>,
                                                     256, 0);
  return e == hipSuccess ? NMX_OK : nmx_fail(NMX_ERR_HIP, "occupancy: %s", hipGetErrorString(e));
}
#endif

extern "C" int nmx_nuts_run_wide(const nmx_nuts_config* cfg, void* arena, float* samples, float* fields,
                                 const int8_t* transform, int model, const float* data, int n, int max_steps,
                                 void* stream) {
  int st = validate(cfg);
  if (st) return st;
  if (!arena) return nmx_fail(NMX_ERR_INVALID, "arena is NULL");
  if (cfg->layout != NMX_LAYOUT_CHAIN_ROWS)
    return nmx_fail(NMX_ERR_INVALID, "run_wide needs the chain-row arena layout (NMX_LAYOUT_CHAIN_ROWS)");
  if (group_count(*cfg) > 1) return nmx_fail(NMX_ERR_INVALID, "run_wide: one chain group only");
  if (cfg->sync_chains)
    return nmx_fail(NMX_ERR_INVALID, "run_wide: per-chain async only (lockstep: one launch per transition)");
  // samples may be NULL: the per-transition fields alone are collected
  if (cfg->collection_size > 0 && (!fields || !transform))
    return nmx_fail(NMX_ERR_INVALID, "collection buffers are NULL");
  if (max_steps <= 0) return nmx_fail(NMX_ERR_INVALID, "run_wide: max_steps must be positive");
  // 32-bit byte offsets within a field
  if ((size_t)cfg->ldc * cfg->dim * 4 > 0xFFFFFFF0ull)
    return nmx_fail(NMX_ERR_INVALID, "run_wide: a vector field exceeds 4 GiB");
  StepArgs args;
  args.a = arena_of(cfg, arena);
  args.cfg = *cfg;
  args.samples = samples;
  args.fields = fields;
  args.transform = transform;
  hipStream_t s = (hipStream_t)stream;
  switch (model) {
    case NMX_WIDE_STOCHASTIC_VOLATILITY:
      if (!data || n <= 1 || n + 2 != cfg->dim)
        return nmx_fail(NMX_ERR_INVALID, "run_wide: stochastic volatility needs returns[T], dim == T + 2");
      return launch_persistent(args, NmxWideSV{data, n}, max_steps, s);
    case NMX_WIDE_FUNNEL:
      if (n != cfg->dim || n < 2) return nmx_fail(NMX_ERR_INVALID, "run_wide: funnel needs n == dim >= 2");
      return launch_persistent(args, NmxWideFunnel{n}, max_steps, s);
    case NMX_WIDE_FUNNEL_NONCENTERED:
      if (n != cfg->dim || n < 2)
        return nmx_fail(NMX_ERR_INVALID, "run_wide: funnel_noncentered needs n == dim >= 2");
      return launch_persistent(args, NmxWideFunnelNC{n}, max_steps, s);
    default:
      return nmx_fail(NMX_ERR_INVALID, "run_wide: unknown model %d", model);
  }
}

