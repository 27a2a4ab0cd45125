// HBM-bound DiT block kernels (gfx950). Every kernel reproduces the rounding points of the
// reference's bf16 PyTorch op sequence (each torch op rounds its result to bf16), so the fused
// kernel returns the same bits as the reference's unfused ops on the same inputs.
//
//   cp25_ln_mod          : [x' = x + gate*y]  ->  LayerNorm(x') * (1 + scale) + shift      (bf16)
//                          minimal_v4_dit.py:1171-1179 (_fn), :1204 / :1237 / :1246 (gated residuals)
//   cp25_final_ln_mod    : fp32-autocast variant for the final layer                         (fp32 out)
//                          minimal_v4_dit.py:974-991
//   cp25_layer_norm      : affine LayerNorm (the cross-view net's layer_norm_cross_view_attn)    (bf16)
//                          predict2_multiview/networks/multiview_cross_dit.py:290, :441
//   cp25_head_rmsnorm_rope: per-head RMSNorm (TE, eps 1e-6) of q and k, optional 3D RoPE in fp32,
//                          result rounded to bf16 as attention() does (minimal_v4_dit.py:410-420,
//                          attention.py:107-109)
//   cp25_gelu            : exact-erf GELU in place (minimal_v4_dit.py:249-254)
//   cp25_patchify        : frame-replace conditioning + mask/padding channels + "(c r m n)" patch
//                          gather (video2world_model_rectified_flow.py:105-107, minimal_v1_lvg_dit.py:46,
//                          minimal_v4_dit.py:1547-1554, :874)
//   cp25_cfg_velocity    : GT-frame velocity replacement + classifier-free guidance, reading the
//                          final layer's token-major output directly ("(p1 p2 t C)" unpatchify)
//                          (video2world_model_rectified_flow.py:131-136, :206-210)
// Token-major layout everywhere: activations are [tokens, B, D] (batch inner), latents are kept in
// "patch layout" [tokens, 64] with index (p1*2+p2)*16 + C, so CP shards are contiguous token ranges.
#include "cp25_common.h"

#pragma clang fp contract(off)

namespace {

// ---------------------------------------------------------------- LayerNorm + modulate
// FP8: h is emitted as the row-scaled fp8 operand of the next (fp8) GEMM instead of bf16: h8_out
// [rows, D] OCP E4M3 and h_scale [rows] = max|h_row| / 448, the same definition as cp25_quant_fp8_rows
// applied to the bf16 h (fp8_ops.hip), without the bf16 h round trip through HBM
template <int NC, bool FP8 = false>  // NC = D / 512 chunks of 8 bf16 per lane
__global__ void __launch_bounds__(256) ln_mod_kernel(
    const unsigned short* __restrict__ x, int64_t x_st, int64_t x_sb,
    const unsigned short* __restrict__ y,  // optional residual branch output [tok, B, D]
    const unsigned short* __restrict__ gate, const unsigned short* __restrict__ shift,
    const unsigned short* __restrict__ scale, int64_t mod_sb, int64_t mod_st,
    unsigned short* __restrict__ x_out, unsigned short* __restrict__ h_out, int64_t n_rows, int B,
    int64_t tok0, int64_t hw, float eps, unsigned char* __restrict__ h8_out = nullptr,
    float* __restrict__ h_scale = nullptr) {
  constexpr int D = NC * 512;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n_rows) return;
  const int64_t tok = row / B;
  const int b = (int)(row % B);
  const int64_t t = (tok0 + tok) / hw;
  const int64_t mo = b * mod_sb + t * mod_st;

  float v[NC * 8];
  const unsigned short* xr = x + tok * x_st + b * x_sb;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    u16x8 w = *reinterpret_cast<const u16x8*>(xr + (c * 64 + lane) * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[c * 8 + e] = bf2f(w[e]);
  }
  if (y != nullptr) {
    const unsigned short* yr = y + row * D;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int off = (c * 64 + lane) * 8;
      u16x8 w = *reinterpret_cast<const u16x8*>(yr + off);
      u16x8 g = *reinterpret_cast<const u16x8*>(gate + mo + off);
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        // x + gate * y : two bf16 torch ops, two roundings
        const float gy = rbf(bf2f(g[e]) * bf2f(w[e]));
        const float xn = rbf(v[c * 8 + e] + gy);
        v[c * 8 + e] = xn;
        o[e] = f2bf(xn);
      }
      *reinterpret_cast<u16x8*>(x_out + row * D + off) = o;
    }
  }
  // two-pass mean / variance in fp32 (torch layer_norm computes bf16 inputs in fp32)
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NC * 8; ++i) s += v[i];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  const float mean = s * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NC * 8; ++i) {
    const float d = v[i] - mean;
    q += d * d;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) q += __shfl_xor(q, m);
  const float rstd = rsqrtf(q * (1.f / D) + eps);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int off = (c * 64 + lane) * 8;
    u16x8 sh = *reinterpret_cast<const u16x8*>(shift + mo + off);
    u16x8 sc = *reinterpret_cast<const u16x8*>(scale + mo + off);
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float ln = rbf((v[c * 8 + e] - mean) * rstd);  // LayerNorm output (bf16 tensor)
      const float one_p = rbf(1.f + bf2f(sc[e]));           // (1 + scale)
      const float prod = rbf(ln * one_p);
      o[e] = f2bf(prod + bf2f(sh[e]));                      // + shift
      if constexpr (FP8) v[c * 8 + e] = bf2f(o[e]);
    }
    if constexpr (!FP8) *reinterpret_cast<u16x8*>(h_out + row * D + off) = o;
  }
  if constexpr (FP8) {
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < NC * 8; ++i) amax = fmaxf(amax, fabsf(v[i]));
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) amax = fmaxf(amax, __shfl_xor(amax, m));
    const float inv = amax > 0.f ? 448.f / amax : 0.f;
    if (lane == 0) h_scale[row] = amax / 448.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      u32x2 o8;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        float f[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) f[e] = fminf(fmaxf(v[c * 8 + 4 * hh + e] * inv, -448.f), 448.f);
        int w = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
        w = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], w, true);
        o8[hh] = (unsigned)w;
      }
      *reinterpret_cast<u32x2*>(h8_out + row * D + (c * 64 + lane) * 8) = o8;
    }
  }
}

// ---------------------------------------------------------------- affine LayerNorm (no modulation)
// nn.LayerNorm(D, elementwise_affine=True, eps) on bf16 rows: fp32 mean / variance (two passes over the registers, as
// ln_mod_kernel), y = (x - mean) * rstd * w + b in fp32, one bf16 rounding (torch's layer_norm on bf16 input and
// weights). One wave per row. The cross-view net's layer_norm_cross_view_attn (multiview_cross_dit.py:290, :441).
template <int NC>
__global__ void __launch_bounds__(256) layer_norm_kernel(const unsigned short* __restrict__ x, int64_t x_stride,
                                                         const unsigned short* __restrict__ w,
                                                         const unsigned short* __restrict__ bias,
                                                         unsigned short* __restrict__ y, int64_t y_stride,
                                                         int64_t n_rows, float eps) {
  constexpr int D = NC * 512;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n_rows) return;
  float v[NC * 8];
  const unsigned short* xr = x + row * x_stride;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    u16x8 t = *reinterpret_cast<const u16x8*>(xr + (c * 64 + lane) * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[c * 8 + e] = bf2f(t[e]);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NC * 8; ++i) s += v[i];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  const float mean = s * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NC * 8; ++i) {
    const float d = v[i] - mean;
    q += d * d;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) q += __shfl_xor(q, m);
  const float rstd = rsqrtf(q * (1.f / D) + eps);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int off = (c * 64 + lane) * 8;
    u16x8 wv = *reinterpret_cast<const u16x8*>(w + off);
    u16x8 bv = *reinterpret_cast<const u16x8*>(bias + off);
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf((v[c * 8 + e] - mean) * rstd * bf2f(wv[e]) + bf2f(bv[e]));
    *reinterpret_cast<u16x8*>(y + row * y_stride + off) = o;
  }
}

// fp32-autocast final-layer variant: LN in fp32, fp32 modulate, fp32 out
template <int NC>
__global__ void __launch_bounds__(256) final_ln_mod_kernel(
    const unsigned short* __restrict__ x, const unsigned short* __restrict__ y,
    const unsigned short* __restrict__ gate, int64_t gmod_sb, int64_t gmod_st,
    const float* __restrict__ shift, const float* __restrict__ scale, int64_t mod_sb, int64_t mod_st,
    float* __restrict__ out, int64_t n_rows, int B, int64_t tok0, int64_t hw, float eps) {
  constexpr int D = NC * 512;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n_rows) return;
  const int64_t tok = row / B;
  const int b = (int)(row % B);
  const int64_t t = (tok0 + tok) / hw;
  float v[NC * 8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int off = (c * 64 + lane) * 8;
    u16x8 w = *reinterpret_cast<const u16x8*>(x + row * D + off);
    if (y != nullptr) {
      u16x8 yy = *reinterpret_cast<const u16x8*>(y + row * D + off);
      u16x8 g = *reinterpret_cast<const u16x8*>(gate + b * gmod_sb + t * gmod_st + off);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[c * 8 + e] = rbf(bf2f(w[e]) + rbf(bf2f(g[e]) * bf2f(yy[e])));
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[c * 8 + e] = bf2f(w[e]);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NC * 8; ++i) s += v[i];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  const float mean = s * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NC * 8; ++i) {
    const float d = v[i] - mean;
    q += d * d;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) q += __shfl_xor(q, m);
  const float rstd = rsqrtf(q * (1.f / D) + eps);
  const int64_t mo = b * mod_sb + t * mod_st;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int off = (c * 64 + lane) * 8;
    f32x4 o0, o1;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float ln = (v[c * 8 + e] - mean) * rstd;
      const float r = ln * (1.f + scale[mo + off + e]) + shift[mo + off + e];
      if (e < 4) o0[e] = r; else o1[e - 4] = r;
    }
    *reinterpret_cast<f32x4*>(out + row * D + off) = o0;
    *reinterpret_cast<f32x4*>(out + row * D + off + 4) = o1;
  }
}

// ---------------------------------------------------------------- per-head RMSNorm (+ RoPE)
// 16 lanes per (row, head) of 128 elements; lane i holds elements 8i .. 8i+7.
// kNmax: also the max |output row| over all (row, head) items into nmax[64 x 32] (atomic max on the float bits into
// slot blockIdx % 64 at float index 32 slot, one atomic per workgroup; the caller zeroes the slots): the data-tight
// key bound of the gated attention
template <bool kNmax = false>
__global__ void __launch_bounds__(256) head_rmsnorm_rope_kernel(
    unsigned short* __restrict__ buf, int64_t row_stride, int64_t n_rows, int B, int H, int head_off,
    const unsigned short* __restrict__ w, const float* __restrict__ cosb, const float* __restrict__ sinb,
    unsigned short* __restrict__ out2, int64_t out2_stride, float eps, float out_scale,
    unsigned int* __restrict__ nmax = nullptr) {
  int64_t item = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);  // (row, head)
  const int li = threadIdx.x & 15;
  const bool valid = item < n_rows * H;
  if constexpr (!kNmax) {
    if (!valid) return;
  } else {
    item = valid ? item : n_rows * H - 1;  // the wave reduction below needs every lane; extra lanes redo the last item
  }
  const int64_t row = item / H;
  const int h = (int)(item % H);
  unsigned short* p = buf + row * row_stride + head_off + h * 128 + li * 8;
  u16x8 raw = *reinterpret_cast<const u16x8*>(p);
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = bf2f(raw[e]);
  float ss = hn_sumsq8(v);  // (the reduction order attn_fwd.hip's in-kernel q normalisation repeats)
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) ss += __shfl_xor(ss, m, 16);
  const float rstd = hn_rstd(ss, eps);
  u16x8 ww = *reinterpret_cast<const u16x8*>(w + li * 8);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = hn_norm(v[e], rstd, bf2f(ww[e]));  // TE RMSNorm -> bf16
  if (cosb != nullptr) {
    // rotate-half RoPE in fp32 (TE fused rope, non-interleaved): y = x*cos + rot(x)*sin
    const int64_t tok = row / B;
    const int dlo = (li & 7) * 8;  // frequency index (freqs repeat with period 64)
    float partner[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) partner[e] = __shfl_xor(v[e], 8, 16);
    const float sgn = li < 8 ? -1.f : 1.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float c = cosb[tok * 64 + dlo + e];
      const float s = sinb[tok * 64 + dlo + e];
      v[e] = hn_rope(v[e], partner[e], sgn, c, s);
    }
  }
  u16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = f2bf(v[e] * out_scale);  // out_scale 1: exact, the reference's rounding
  if constexpr (kNmax) {
    float nn = 0.f;  // |row|^2 of the bf16 values written (the ones the attention reads)
#pragma unroll
    for (int e = 0; e < 8; ++e) nn = fmaf(bf2f(o[e]), bf2f(o[e]), nn);
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) nn += __shfl_xor(nn, m, 16);  // the item's 16 lanes
    nn = fmaxf(nn, __shfl_xor(nn, 16));                             // the wave's 4 items
    nn = fmaxf(nn, __shfl_xor(nn, 32));
    __shared__ float wmax[4];
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = nn;
    __syncthreads();
    // one atomic per workgroup, into one of 64 slots a cache line apart (all slots in one line serialised the
    // atomics of the whole launch on one L2 channel: ~3.5 ms per launch at the DiT shape)
    if (threadIdx.x == 0)
      atomicMax(nmax + (blockIdx.x & 63) * 32, __float_as_uint(sqrtf(fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3])))));
  }
  if (!kNmax || valid) {
    *reinterpret_cast<u16x8*>(p) = o;
    if (out2 != nullptr) *reinterpret_cast<u16x8*>(out2 + row * out2_stride + h * 128 + li * 8) = o;
  }
}

// plain strided copy of a [rows, width] bf16 block (K/V export for the CP all-gather)
__global__ void __launch_bounds__(256) copy_rows_kernel(const unsigned short* __restrict__ src, int64_t src_stride,
                                                        unsigned short* __restrict__ dst, int64_t dst_stride,
                                                        int64_t n_rows, int width8) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_rows * width8) return;
  const int64_t r = i / width8;
  const int c = (int)(i % width8);
  *reinterpret_cast<u16x8*>(dst + r * dst_stride + c * 8) = *reinterpret_cast<const u16x8*>(src + r * src_stride + c * 8);
}

// ---------------------------------------------------------------- GELU (exact erf)
__global__ void __launch_bounds__(256) gelu_kernel(unsigned short* __restrict__ x, int64_t n8) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  u16x8 w = *reinterpret_cast<const u16x8*>(x + i * 8);
  u16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float a = bf2f(w[e]);
    o[e] = f2bf(gelu_erf(a));
  }
  *reinterpret_cast<u16x8*>(x + i * 8) = o;
}

// ---------------------------------------------------------------- patchify
// state / gt in patch layout [tok, 64] (index p*16 + c, p = p1*2 + p2); out [tok, 72] bf16 with
// feature index c*4 + p for c in 0..17 (16 latent channels, condition mask, padding mask).
__global__ void __launch_bounds__(256) patchify_kernel(const float* __restrict__ xs, const float* __restrict__ gt,
                                                       const float* __restrict__ frame_mask,
                                                       const unsigned short* __restrict__ pad_mask,
                                                       unsigned short* __restrict__ out, int64_t out_ld,
                                                       int64_t n_tok, int64_t tok0, int64_t hw) {
  const int64_t tok = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int j = threadIdx.x & 63;  // j = p*16 + c
  if (tok >= n_tok) return;
  const float m = frame_mask[(tok0 + tok) / hw];
  const int p = j >> 4, c = j & 15;
  const float x = xs[tok * 64 + j];
  float xin;
  if (gt != nullptr) {
    const float a = gt[tok * 64 + j] * m;
    const float bb = 1.f - m;
    xin = a + x * bb;  // gt*mask + xt*(1-mask)
  } else {
    xin = x;
  }
  unsigned short* o = out + tok * out_ld;
  o[c * 4 + p] = f2bf(xin);
  if (j < 4) {
    o[64 + j] = f2bf(m);
    o[68 + j] = pad_mask != nullptr ? pad_mask[tok * 4 + j] : (unsigned short)0;
  }
  for (int64_t z = 72 + j; z < out_ld; z += 64) o[z] = 0;  // a padded row (the own GEMM's K = 128): zero columns
}

// ---------------------------------------------------------------- GT velocity + CFG
// net: final-layer output [tok, B, 64] fp32 (feature index (p1*2+p2)*16 + C == patch layout).
__global__ void __launch_bounds__(256) cfg_velocity_kernel(const float* __restrict__ net, int B,
                                                           const float* __restrict__ noise, const float* __restrict__ gt,
                                                           const float* __restrict__ frame_mask, float guidance,
                                                           int cfg_mode, float* __restrict__ v_out, int64_t n_tok,
                                                           int64_t tok0, int64_t hw) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_tok * 64) return;
  const int64_t tok = i >> 6;
  const int j = (int)(i & 63);
  float vb[2];
  const float m = gt != nullptr ? frame_mask[(tok0 + tok) / hw] : 0.f;
  for (int b = 0; b < B && b < 2; ++b) {
    const float n = net[(tok * B + b) * 64 + j];
    if (gt != nullptr) {
      const float gv = noise[i] - gt[i];   // gt_frames_velocity = noise - gt
      const float a = gv * m;
      const float bb = 1.f - m;
      const float c = n * bb;
      vb[b] = a + c;
    } else {
      vb[b] = n;
    }
  }
  float v;
  if (B == 1) {
    v = vb[0];
  } else if (cfg_mode == 0) {
    v = vb[0] + guidance * (vb[0] - vb[1]);  // Video2World: cond + g (cond - uncond)
  } else {
    v = vb[1] + guidance * (vb[0] - vb[1]);  // Text2World: uncond + g (cond - uncond)
  }
  v_out[i] = v;
}

}  // namespace

// ============================================================================ C ABI
namespace {
template <bool FP8>
int launch_ln_mod(const void* x, int64_t x_st, int64_t x_sb, const void* y, const void* gate, const void* shift,
                  const void* scale, int64_t mod_sb, int64_t mod_st, void* x_out, void* h_out, void* h8_out,
                  float* h_scale, int64_t n_tok, int B, int D, int64_t tok0, int64_t hw, float eps,
                  hipStream_t stream) {
  if (n_tok <= 0 || B <= 0 || hw <= 0 || !x || !shift || !scale) return CP25_ERR_INVAL;
  if (FP8 ? (!h8_out || !h_scale) : !h_out) return CP25_ERR_INVAL;
  if (y != nullptr && (gate == nullptr || x_out == nullptr)) return CP25_ERR_INVAL;
  const int64_t rows = n_tok * B;
  const dim3 grid((unsigned)cdiv(rows, 4));
  auto* X = (const unsigned short*)x;
  auto* Y = (const unsigned short*)y;
  auto* G = (const unsigned short*)gate;
  auto* SH = (const unsigned short*)shift;
  auto* SC = (const unsigned short*)scale;
  auto* XO = (unsigned short*)x_out;
  auto* HO = (unsigned short*)h_out;
  auto* H8 = (unsigned char*)h8_out;
#define LNM(NC) hipLaunchKernelGGL((ln_mod_kernel<NC, FP8>), grid, dim3(256), 0, stream, X, x_st, x_sb, Y, G, SH, SC, mod_sb, mod_st, XO, HO, rows, B, tok0, hw, eps, H8, h_scale)
  switch (D) {
    case 512: LNM(1); break;
    case 1024: LNM(2); break;
    case 2048: LNM(4); break;
    case 4096: LNM(8); break;
    case 5120: LNM(10); break;
    default: return CP25_ERR_DTYPE;
  }
#undef LNM
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}
}  // namespace

extern "C" int cp25_ln_mod(const void* x, int64_t x_st, int64_t x_sb, const void* y, const void* gate,
                           const void* shift, const void* scale, int64_t mod_sb, int64_t mod_st, void* x_out,
                           void* h_out, int64_t n_tok, int B, int D, int64_t tok0, int64_t hw, float eps,
                           hipStream_t stream) {
  return launch_ln_mod<false>(x, x_st, x_sb, y, gate, shift, scale, mod_sb, mod_st, x_out, h_out, nullptr, nullptr,
                              n_tok, B, D, tok0, hw, eps, stream);
}

extern "C" int cp25_ln_mod_fp8(const void* x, int64_t x_st, int64_t x_sb, const void* y, const void* gate,
                               const void* shift, const void* scale, int64_t mod_sb, int64_t mod_st, void* x_out,
                               void* h8_out, float* h_scale, int64_t n_tok, int B, int D, int64_t tok0, int64_t hw,
                               float eps, hipStream_t stream) {
  return launch_ln_mod<true>(x, x_st, x_sb, y, gate, shift, scale, mod_sb, mod_st, x_out, nullptr, h8_out, h_scale,
                             n_tok, B, D, tok0, hw, eps, stream);
}

extern "C" int cp25_final_ln_mod(const void* x, const void* y, const void* gate, int64_t gmod_sb, int64_t gmod_st,
                                 const float* shift, const float* scale, int64_t mod_sb, int64_t mod_st, float* out,
                                 int64_t n_tok, int B, int D, int64_t tok0, int64_t hw, float eps, hipStream_t stream) {
  if (n_tok <= 0 || B <= 0 || hw <= 0 || !x || !shift || !scale || !out) return CP25_ERR_INVAL;
  if (y != nullptr && gate == nullptr) return CP25_ERR_INVAL;
  const int64_t rows = n_tok * B;
  const dim3 grid((unsigned)cdiv(rows, 4));
  auto* X = (const unsigned short*)x;
  auto* Y = (const unsigned short*)y;
  auto* G = (const unsigned short*)gate;
#define FLN(NC) hipLaunchKernelGGL(final_ln_mod_kernel<NC>, grid, dim3(256), 0, stream, X, Y, G, gmod_sb, gmod_st, shift, scale, mod_sb, mod_st, out, rows, B, tok0, hw, eps)
  switch (D) {
    case 512: FLN(1); break;
    case 1024: FLN(2); break;
    case 2048: FLN(4); break;
    case 4096: FLN(8); break;
    case 5120: FLN(10); break;
    default: return CP25_ERR_DTYPE;
  }
#undef FLN
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

extern "C" int cp25_layer_norm(const void* x, int64_t x_stride, const void* weight, const void* bias, void* y,
                               int64_t y_stride, int64_t n_rows, int D, float eps, hipStream_t stream) {
  if (!x || !weight || !bias || !y || n_rows <= 0 || x_stride < D || y_stride < D) return CP25_ERR_INVAL;
  if ((x_stride % 8) || (y_stride % 8) || (((uintptr_t)x | (uintptr_t)y | (uintptr_t)weight | (uintptr_t)bias) & 15))
    return CP25_ERR_INVAL;
  const dim3 grid((unsigned)cdiv(n_rows, 4));
  auto* X = (const unsigned short*)x;
  auto* W = (const unsigned short*)weight;
  auto* Bi = (const unsigned short*)bias;
  auto* Y = (unsigned short*)y;
#define LNA(NC) hipLaunchKernelGGL(layer_norm_kernel<NC>, grid, dim3(256), 0, stream, X, x_stride, W, Bi, Y, y_stride, n_rows, eps)
  switch (D) {
    case 512: LNA(1); break;
    case 1024: LNA(2); break;
    case 2048: LNA(4); break;
    case 4096: LNA(8); break;
    case 5120: LNA(10); break;
    default: return CP25_ERR_DTYPE;
  }
#undef LNA
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

extern "C" int cp25_head_rmsnorm_rope(void* buf, int64_t row_stride, int64_t n_rows, int B, int H, int head_off,
                                      const void* weight, const float* cos_tab, const float* sin_tab, void* out2,
                                      int64_t out2_stride, float eps, hipStream_t stream) {
  return cp25_head_rmsnorm_rope_scaled(buf, row_stride, n_rows, B, H, head_off, weight, cos_tab, sin_tab, out2,
                                       out2_stride, eps, 1.f, stream);
}

extern "C" int cp25_head_rmsnorm_rope_scaled(void* buf, int64_t row_stride, int64_t n_rows, int B, int H,
                                             int head_off, const void* weight, const float* cos_tab,
                                             const float* sin_tab, void* out2, int64_t out2_stride, float eps,
                                             float out_scale, hipStream_t stream) {
  return cp25_head_rmsnorm_rope_nmax(buf, row_stride, n_rows, B, H, head_off, weight, cos_tab, sin_tab, out2,
                                     out2_stride, eps, out_scale, nullptr, stream);
}

extern "C" int cp25_head_rmsnorm_rope_nmax(void* buf, int64_t row_stride, int64_t n_rows, int B, int H, int head_off,
                                           const void* weight, const float* cos_tab, const float* sin_tab, void* out2,
                                           int64_t out2_stride, float eps, float out_scale, float* norm_max_slots,
                                           hipStream_t stream) {
  if (!buf || !weight || n_rows <= 0 || H <= 0 || B <= 0) return CP25_ERR_INVAL;
  if ((row_stride % 8) || (head_off % 8) || ((cos_tab == nullptr) != (sin_tab == nullptr))) return CP25_ERR_INVAL;
  if ((uintptr_t)norm_max_slots & 3) return CP25_ERR_INVAL;
  const int64_t items = n_rows * H;
  if (norm_max_slots)
    hipLaunchKernelGGL(head_rmsnorm_rope_kernel<true>, dim3((unsigned)cdiv(items, 16)), dim3(256), 0, stream,
                       (unsigned short*)buf, row_stride, n_rows, B, H, head_off, (const unsigned short*)weight, cos_tab,
                       sin_tab, (unsigned short*)out2, out2_stride, eps, out_scale, (unsigned int*)norm_max_slots);
  else
    hipLaunchKernelGGL(head_rmsnorm_rope_kernel<false>, dim3((unsigned)cdiv(items, 16)), dim3(256), 0, stream,
                       (unsigned short*)buf, row_stride, n_rows, B, H, head_off, (const unsigned short*)weight, cos_tab,
                       sin_tab, (unsigned short*)out2, out2_stride, eps, out_scale, nullptr);
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

extern "C" int cp25_copy_rows(const void* src, int64_t src_stride, void* dst, int64_t dst_stride, int64_t n_rows,
                              int64_t width, hipStream_t stream) {
  if (!src || !dst || n_rows <= 0 || width <= 0 || (width % 8) || (src_stride % 8) || (dst_stride % 8))
    return CP25_ERR_INVAL;
  const int64_t n = n_rows * (width / 8);
  hipLaunchKernelGGL(copy_rows_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream,
                     (const unsigned short*)src, src_stride, (unsigned short*)dst, dst_stride, n_rows, (int)(width / 8));
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

extern "C" int cp25_gelu(void* x, int64_t n, hipStream_t stream) {
  if (!x || n <= 0 || (n % 8)) return CP25_ERR_INVAL;
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(gelu_kernel, dim3((unsigned)cdiv(n8, 256)), dim3(256), 0, stream, (unsigned short*)x, n8);
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

extern "C" int cp25_patchify(const float* xs, const float* gt, const float* frame_mask, const void* pad_mask, void* out,
                             int64_t n_tok, int64_t tok0, int64_t hw, hipStream_t stream) {
  if (!xs || !frame_mask || !out || n_tok <= 0 || hw <= 0) return CP25_ERR_INVAL;
  hipLaunchKernelGGL(patchify_kernel, dim3((unsigned)cdiv(n_tok, 4)), dim3(256), 0, stream, xs, gt, frame_mask,
                     (const unsigned short*)pad_mask, (unsigned short*)out, (int64_t)72, n_tok, tok0, hw);
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

extern "C" int cp25_patchify_ld(const float* xs, const float* gt, const float* frame_mask, const void* pad_mask,
                                void* out, int64_t out_ld, int64_t n_tok, int64_t tok0, int64_t hw, hipStream_t stream) {
  if (!xs || !frame_mask || !out || n_tok <= 0 || hw <= 0 || out_ld < 72 || out_ld % 8) return CP25_ERR_INVAL;
  hipLaunchKernelGGL(patchify_kernel, dim3((unsigned)cdiv(n_tok, 4)), dim3(256), 0, stream, xs, gt, frame_mask,
                     (const unsigned short*)pad_mask, (unsigned short*)out, out_ld, n_tok, tok0, hw);
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

extern "C" int cp25_cfg_velocity(const float* net, int B, const float* noise, const float* gt, const float* frame_mask,
                                 float guidance, int cfg_mode, float* v_out, int64_t n_tok, int64_t tok0, int64_t hw,
                                 hipStream_t stream) {
  if (!net || !v_out || n_tok <= 0 || B < 1 || B > 2 || hw <= 0) return CP25_ERR_INVAL;
  if (gt != nullptr && (noise == nullptr || frame_mask == nullptr)) return CP25_ERR_INVAL;
  const int64_t n = n_tok * 64;
  hipLaunchKernelGGL(cfg_velocity_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, net, B, noise, gt,
                     frame_mask, guidance, cfg_mode, v_out, n_tok, tok0, hw);
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}
