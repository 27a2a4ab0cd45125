// Fused UniPC (bh2, flow prediction, predict_x0) sampler update for gfx950.
//
// One launch per sampler step replaces the elementwise part of
// FlowUniPCMultistepScheduler.step (cosmos_predict2/_src/predict2/models/fm_solvers_unipc.py:630-713):
//   convert_model_output  (:301-318)   x0 = sample - sigma * v
//   multistep_uni_c_bh_update (:466-601, corrector, order 1 or 2)
//   history shift + multistep_uni_p_bh_update (:337-464, predictor, order 1 or 2)
// The scalar coefficients (sigma ratios, h_phi_1, B_h, rhos, 1/rk) are computed on the host with the
// reference's own fp32 torch op sequence; here every tensor op of the reference is one IEEE fp32
// operation in the same order (FP contraction is off), so the update is bit-exact.
// Division of a CUDA tensor by a CPU 0-dim tensor runs as a multiply by the fp32 reciprocal in
// PyTorch (BinaryDivTrueKernel.cu), so D1 = (m_i - m_0) * inv_rk.
#include "cp25_common.h"

#pragma clang fp contract(off)

// cp25_unipc_params: see include/cp25.h

namespace {
__global__ void __launch_bounds__(256) unipc_kernel(float* __restrict__ x, const float* __restrict__ v,
                                                    float* __restrict__ m0, float* __restrict__ m1,
                                                    float* __restrict__ last, int64_t n, cp25_unipc_params P) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float xi = x[i];
  const float sv = P.sigma * v[i];
  const float mc = xi - sv;  // model_output_convert
  const float m0o = m0[i];
  if (P.use_corr) {
    const float t1 = P.c_a * last[i];
    const float t2 = P.c_b * m0o;
    const float xt_ = t1 - t2;
    const float d1t = mc - m0o;
    float s;
    if (P.order_c == 2) {
      const float d1 = (m1[i] - m0o) * P.c_inv_rk;
      const float corr = P.c_rho0 * d1;
      s = corr + P.c_rho_last * d1t;
    } else {
      s = P.c_rho_last * d1t;
    }
    xi = xt_ - P.c_c * s;
  }
  // history: model_outputs[-2] <- old m0, model_outputs[-1] <- mc ; last_sample <- xi
  const float pa = P.p_a * xi;
  const float pb = P.p_b * mc;
  float xp = pa - pb;
  if (P.order_p == 2) {
    const float d1 = (m0o - mc) * P.p_inv_rk;
    const float pred = P.p_rho0 * d1;
    xp = xp - P.p_c * pred;
  }
  x[i] = xp;
  m1[i] = m0o;
  m0[i] = mc;
  last[i] = xi;
}
}  // namespace

extern "C" int cp25_unipc_step(float* x, const float* v, float* m0, float* m1, float* last, int64_t n,
                               const cp25_unipc_params* params, hipStream_t stream) {
  if (!x || !v || !m0 || !m1 || !last || !params || n <= 0) return CP25_ERR_INVAL;
  const cp25_unipc_params P = *params;
  if ((P.order_c != 1 && P.order_c != 2) || (P.order_p != 1 && P.order_p != 2)) return CP25_ERR_INVAL;
  hipLaunchKernelGGL(unipc_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, x, v, m0, m1, last, n, P);
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}
