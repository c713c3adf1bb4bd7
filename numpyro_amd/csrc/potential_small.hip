// Potentials of small-D models: one thread per chain, coordinates loop in registers
// (per-chain bodies in nmx_small_models.h, shared with the persistent NUTS kernel).
#include <math.h>

#include "nmx_api_internal.h"
#include "nmx_common.h"
#include "nmx_small_models.h"

namespace {

__global__ void k_diag_normal(const float* mu, const float* prec, int D, nmx_eval_batch ev) {
  const int c = nmx_eval_chain(ev, blockIdx.x * blockDim.x + threadIdx.x);
  if (c < 0) return;
  NmxDiagNormal{mu, prec, D}(ev, c);
}

__global__ void k_eight_schools(const float* y, const float* sigma, int J, nmx_eval_batch ev) {
  const int c = nmx_eval_chain(ev, blockIdx.x * blockDim.x + threadIdx.x);
  if (c < 0) return;
  NmxEightSchools{y, sigma, J}(ev, c);
}

int check_ev(const nmx_eval_batch* ev) {
  if (!ev || !ev->z || !ev->grad || !ev->pe) return nmx_fail(NMX_ERR_INVALID, "eval batch has NULL pointers");
  if (ev->num_chains <= 0 || ev->ldc < ev->num_chains)
    return nmx_fail(NMX_ERR_INVALID, "bad num_chains/ldc (%d/%d)", ev->num_chains, ev->ldc);
  return NMX_OK;
}

}  // namespace

extern "C" int nmx_pe_diag_normal(const float* mu, const float* prec, int dim, const nmx_eval_batch* ev,
                                  void* stream) {
  if (int st = check_ev(ev)) return st;
  if (!mu || !prec || dim <= 0) return nmx_fail(NMX_ERR_INVALID, "bad diag_normal parameters");
  hipLaunchKernelGGL(k_diag_normal, dim3((ev->num_chains + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     mu, prec, dim, *ev);
  return nmx_check_launch("k_diag_normal");
}

extern "C" int nmx_pe_eight_schools(const float* y, const float* sigma, int J, const nmx_eval_batch* ev,
                                    void* stream) {
  if (int st = check_ev(ev)) return st;
  if (!y || !sigma || J <= 0) return nmx_fail(NMX_ERR_INVALID, "bad eight_schools data");
  hipLaunchKernelGGL(k_eight_schools, dim3((ev->num_chains + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     y, sigma, J, *ev);
  return nmx_check_launch("k_eight_schools");
}
