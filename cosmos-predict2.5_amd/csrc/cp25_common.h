// Shared device/host helpers for the cosmos-predict2.5 MI355X kernels (gfx950 only).
//
// Conventions used by every entry point in include/cp25.h:
//   * tensors are device pointers + element strides; the caller (PyTorch's caching
//     allocator on the Python side) owns all memory, kernels never allocate;
//   * every call is stream-ordered on the hipStream_t passed in, never synchronises,
//     and is safe to capture into a hipGraph;
//   * return 0 on success, a negative errno-style code on bad arguments (checked on the
//     host before any launch), or CP25_ERR_LAUNCH if the launch itself failed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "cp25.h"

#define CP25_OK 0
#define CP25_ERR_INVAL (-22)   /* bad shape / stride / size */
#define CP25_ERR_DTYPE (-95)   /* unsupported dtype / head dim */
#define CP25_ERR_LAUNCH (-5)   /* hipLaunch failure */

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// bf16 <-> f32 with round-to-nearest-even (matches torch's .to(bfloat16)).
__device__ __forceinline__ float bf2f(unsigned short b) { return __uint_as_float(((unsigned)b) << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
  // plain conversion: hipcc lowers it to v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950
  __bf16 h = static_cast<__bf16>(f);
  return __builtin_bit_cast(unsigned short, h);
}
// round an f32 to the nearest bf16 value and return it as f32 (emulates a bf16 tensor op)
__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }

// Per-head RMSNorm (TE, over 128 elements) + rotate-half RoPE, piece by piece: cp25_head_rmsnorm_rope's arithmetic,
// shared by its kernel (dit_ops.hip) and the self-attention's in-kernel q normalisation (attn_fwd.hip), which reduce
// the 16 8-element partial sums in the same order, so the two give the same bits. FP contraction off in each piece
// (the attention's translation unit contracts by default).
__device__ __forceinline__ float hn_sumsq8(const float* x) {  // x[0..7] sequentially
#pragma clang fp contract(off)
  float ss = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) ss += x[e] * x[e];
  return ss;
}
__device__ __forceinline__ float hn_rstd(float ss, float eps) {
#pragma clang fp contract(off)
  return rsqrtf(ss * (1.f / 128.f) + eps);
}
__device__ __forceinline__ float hn_norm(float x, float rstd, float w) {  // TE RMSNorm output -> bf16 value
#pragma clang fp contract(off)
  return rbf((x * rstd) * w);
}
__device__ __forceinline__ float hn_rope(float v, float partner, float sgn, float c, float s) {  // x cos + rot(x) sin
#pragma clang fp contract(off)
  return fmaf(v, c, (sgn * partner) * s);
}

// Exact-erf GELU, x * Phi(x) (minimal_v4_dit.py:249-254, nn.GELU()), with Phi from one erfc evaluation:
// z = |x| / sqrt(2), erfc(z) = (1 + p(q)) / (1 + 2 z) * exp(-z^2), q = (z - 2) / (z + 2), p the degree-9 fit of
// (1 + 2 z) exp(z^2) erfc(z) - 1 on z in [0, 10.5] (4.7e-8 relative; the construction of Juffa's erfcf), and
// Phi(x >= 0) = 1 - erfc / 2, Phi(x < 0) = erfc / 2 taken directly (no 1 + erf cancellation for negative x).
// Branch-free, two v_rcp_f32 and one v_exp_f32 against libm erff's ~39 ops with two paths: the GEMM epilogue
// runs it on 1.8e9 values per MLP. Within 8e-6 relative of the float64 GELU for |x| < 9; rounded to bf16 it
// differs from the correctly rounded value on 1.4e-5 of N(0, 1.5^2) inputs (by one ulp; libm-level accuracy).
__device__ __forceinline__ float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float q = (z - 2.f) * __builtin_amdgcn_rcpf(z + 2.f);
  float p = -0x1.9d90e0p-12f;
  p = fmaf(p, q, -0x1.408798p-10f);
  p = fmaf(p, q, 0x1.56ecf8p-10f);
  p = fmaf(p, q, 0x1.1a9db8p-7f);
  p = fmaf(p, q, -0x1.080d7ap-7f);
  p = fmaf(p, q, -0x1.bc0636p-5f);
  p = fmaf(p, q, 0x1.4ffc24p-3f);
  p = fmaf(p, q, -0x1.540864p-3f);
  p = fmaf(p, q, -0x1.7bf612p-4f);
  p = fmaf(p, q, 0x1.1ba03ap-2f);
  const float ec = (1.f + p) * __builtin_amdgcn_rcpf(fmaf(2.f, z, 1.f)) *
                   __builtin_amdgcn_exp2f(-(z * z) * 1.44269504088896340736f);
  return x * (x >= 0.f ? fmaf(-0.5f, ec, 1.f) : 0.5f * ec);
}

__host__ __device__ __forceinline__ int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// XCD-aware bijective remap of a 1-D grid: blocks b and b+8 share an XCD, so give each
// group of 8 a contiguous range of logical tiles (cdna_hip_programming.md §5 T1).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

#define CP25_LAUNCH_CHECK()                                     \
  do {                                                          \
    if (hipGetLastError() != hipSuccess) return CP25_ERR_LAUNCH; \
  } while (0)
