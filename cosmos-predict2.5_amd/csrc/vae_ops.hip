// Wan2.1 causal video VAE kernels (gfx950), channels-last activations [frame][h][w][C] bf16.
//
//   cp25_conv3d       : implicit-GEMM causal Conv3d / Conv2d with bf16 MFMA (v_mfma_f32_32x32x16_bf16),
//                       replacing torch conv3d/conv2d (cuDNN) in CausalConv3d (tokenizers/wan2pt1.py:44-62),
//                       Resample (:88-162: nearest 2x upsample fused into the input gather, stride-2
//                       downsample with ZeroPad2d((0,1,0,1)), (3,1,1) time_conv with the frame
//                       interleave of :139-141 fused into the epilogue), the 1x1 shortcut/conv1/conv2,
//                       and the AttentionBlock 1x1 projections (:236-237). Bias and the residual add
//                       (ResidualBlock :222, AttentionBlock :261) are fused into the epilogue with the
//                       reference's bf16 rounding points (conv output rounded, then x + h rounded).
//   cp25_rms_norm_silu: RMS_norm (F.normalize over C * sqrt(C) * gamma, :65-77) [+ SiLU], per pixel.
//
// Causality: the temporal taps read a table of frame pointers [zero-pad | cached frames | new frames]
// built by the host from the reference's feat_cache rules, so no padded copy of the clip is made.
// GEMM view: D[cout][pixel] = W[cout][k] * X[k][pixel], k = (kt, kh, kw, cin); the pixel is on the
// MFMA lane so the epilogue writes 4 contiguous channels (8 B) per lane.
#include "cp25_common.h"

namespace {

constexpr int kMaxFrames = 24;
constexpr int kBM = 128;  // output pixels per workgroup (4 waves x 32)

struct ConvArgs {
  const unsigned short* frames[kMaxFrames];  // input frames [Hin][Win][Cin]; nullptr = zeros
  int n_frames;
  const unsigned short* w;  // [Cout][KT][KH][KW][Cin]
  const unsigned short* bias;  // [Cout] bf16 or nullptr
  const unsigned short* residual;  // same layout as out or nullptr
  unsigned short* out;  // [Tout][Ho][Wo][Cout] (or interleaved, see out_split)
  int Hin, Win, Cin, Ho, Wo, Cout, Tout;
  int KT, KH, KW;
  int stride_t, stride_hw, pad_top, pad_left;
  int upsample;  // 1: input is nearest-2x upsampled (pad applies in upsampled coords)
  int out_split;  // >0: cout >= out_split goes to frame 2*to+1 channel cout-out_split (frame interleave)
  int out_C;      // channels of the output tensor (Cout, or out_split when interleaving)
};

template <int BK>
__device__ __forceinline__ int a_swz(int row, int chunk) {
  constexpr int cpr = BK / 8;          // 16-B chunks per LDS row
  constexpr int rpb = 16 / cpr;        // rows per 256-B bank row
  return chunk ^ ((row / rpb) & (cpr - 1));
}

template <int BK, int NT>
__global__ void __launch_bounds__(256) conv_igemm_kernel(ConvArgs a) {
  constexpr int BN = 32 * NT;
  constexpr int CPR = BK / 8;  // chunks per row
  constexpr int A_BYTES = kBM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_CHUNKS = kBM * CPR;
  constexpr int B_CHUNKS = BN * CPR;
  constexpr int A_PER_T = (A_CHUNKS + 255) / 256;
  constexpr int B_PER_T = (B_CHUNKS + 255) / 256;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l31 = lane & 31, hl = lane >> 5;
  const int m0 = blockIdx.x * kBM;
  const int n0 = blockIdx.y * BN;
  const int to = blockIdx.z;
  const int M = a.Ho * a.Wo;
  const int K = a.KT * a.KH * a.KW * a.Cin;
  const int kc_per_tap = a.Cin / BK;
  const int nk = a.KT * a.KH * a.KW * kc_per_tap;

  // per-thread A rows (pixels) this thread stages: their output coordinates are fixed for the whole
  // K loop, so the pixel -> (ho, wo) division and the padding offsets are done once here; a k-step
  // only adds its tap (kh, kw)
  u32x4 ra[A_PER_T], rb[B_PER_T];
  int a_h0[A_PER_T], a_w0[A_PER_T], a_off[A_PER_T];
#pragma unroll
  for (int i = 0; i < A_PER_T; ++i) {
    const int c = tid + 256 * i;
    const int row = c / CPR, ch = c % CPR;
    const int p = m0 + row;
    a_off[i] = ch * 8;
    if (c < A_CHUNKS && p < M) {
      const int ho = p / a.Wo, wo = p % a.Wo;
      a_h0[i] = a.upsample ? ho - a.pad_top : ho * a.stride_hw - a.pad_top;
      a_w0[i] = a.upsample ? wo - a.pad_left : wo * a.stride_hw - a.pad_left;
    } else {
      a_h0[i] = -(1 << 28);  // never in range
      a_w0[i] = 0;
    }
  }

  auto load_stage = [&](int ks) {
    const int tap = ks / kc_per_tap;
    const int c0 = (ks % kc_per_tap) * BK;
    const int kw = tap % a.KW;
    const int kh = (tap / a.KW) % a.KH;
    const int kt = tap / (a.KW * a.KH);
    const int fi = to * a.stride_t + kt;
    const unsigned short* fr = (fi < a.n_frames) ? a.frames[fi] : nullptr;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      u32x4 v = {0u, 0u, 0u, 0u};
      if (fr != nullptr) {
        int hi, wi;
        bool ok;
        if (a.upsample) {
          const int hu = a_h0[i] + kh, wu = a_w0[i] + kw;
          ok = hu >= 0 && hu < 2 * a.Hin && wu >= 0 && wu < 2 * a.Win;
          hi = hu >> 1;
          wi = wu >> 1;
        } else {
          hi = a_h0[i] + kh;
          wi = a_w0[i] + kw;
          ok = hi >= 0 && hi < a.Hin && wi >= 0 && wi < a.Win;
        }
        if (ok) v = *reinterpret_cast<const u32x4*>(fr + ((int64_t)hi * a.Win + wi) * a.Cin + c0 + a_off[i]);
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int c = tid + 256 * i;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (c < B_CHUNKS) {
        const int row = c / CPR, ch = c % CPR;
        const int co = n0 + row;
        if (co < a.Cout) v = *reinterpret_cast<const u32x4*>(a.w + (int64_t)co * K + tap * a.Cin + c0 + ch * 8);
      }
      rb[i] = v;
    }
  };
  auto store_stage = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int c = tid + 256 * i;
      if (c < A_CHUNKS) {
        const int row = c / CPR, ch = c % CPR;
        *reinterpret_cast<u32x4*>(As + row * BK * 2 + 16 * a_swz<BK>(row, ch)) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int c = tid + 256 * i;
      if (c < B_CHUNKS) {
        const int row = c / CPR, ch = c % CPR;
        *reinterpret_cast<u32x4*>(Bs + row * BK * 2 + 16 * a_swz<BK>(row, ch)) = rb[i];
      }
    }
  };

  f32x16 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  load_stage(0);
  store_stage(0);
  __syncthreads();
  const int prow = wave * 32 + l31;  // this lane's pixel row in the A tile
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) load_stage(ks + 1);
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int ch = 2 * s + hl;
      const bf16x8 xf = *reinterpret_cast<const bf16x8*>(As + prow * BK * 2 + 16 * a_swz<BK>(prow, ch));
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int crow = j * 32 + l31;
        const bf16x8 wf = *reinterpret_cast<const bf16x8*>(Bs + crow * BK * 2 + 16 * a_swz<BK>(crow, ch));
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, xf, acc[j], 0, 0, 0);
      }
    }
    if (ks + 1 < nk) store_stage(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane = pixel, regs = 4-channel groups
  const int p = m0 + prow;
  if (p >= M) return;
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int co = n0 + j * 32 + 8 * g + 4 * hl;
      if (co >= a.Cout) continue;
      int ofr = to, och = co;
      if (a.out_split > 0) {
        ofr = 2 * to + (co >= a.out_split);
        och = co % a.out_split;
      }
      unsigned short* op = a.out + ((int64_t)ofr * M + p) * a.out_C + och;
      const int nvalid = min(4, a.Cout - co);
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = acc[j][4 * g + e];
        if (a.bias != nullptr && e < nvalid) x += bf2f(a.bias[co + e]);
        v[e] = rbf(x);
      }
      if (a.residual != nullptr) {
        const unsigned short* rp = a.residual + ((int64_t)ofr * M + p) * a.out_C + och;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (e < nvalid) v[e] = rbf(v[e] + bf2f(rp[e]));
      }
      if (nvalid == 4 && (a.out_C % 4) == 0) {
        u16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = f2bf(v[e]);
        *reinterpret_cast<u16x4*>(op) = w;
      } else {
        for (int e = 0; e < nvalid; ++e) op[e] = f2bf(v[e]);
      }
    }
}

// ---------------------------------------------------------------- RMS_norm (+ SiLU), channels-last
// 4 lanes per pixel, each lane C/32 vectors of 8 channels (C in {32, 64, 96, ..., 384, ...}).
template <int VPL>
__global__ void __launch_bounds__(256) rms_norm_silu_kernel(const unsigned short* __restrict__ x,
                                                            const unsigned short* __restrict__ gamma,
                                                            unsigned short* __restrict__ y, int64_t n_pix,
                                                            float scale, int do_silu) {
  constexpr int C = VPL * 32;
  const int64_t pix = (int64_t)blockIdx.x * 64 + (threadIdx.x >> 2);
  const int q = threadIdx.x & 3;
  if (pix >= n_pix) return;
  const unsigned short* xr = x + pix * C;
  float v[VPL * 8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    u16x8 w = *reinterpret_cast<const u16x8*>(xr + (i * 4 + q) * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[i * 8 + e] = bf2f(w[e]);
      ss += v[i * 8 + e] * v[i * 8 + e];
    }
  }
  ss += __shfl_xor(ss, 1, 4);
  ss += __shfl_xor(ss, 2, 4);
  // F.normalize: x / max(||x||, 1e-12) with ||x|| a bf16 tensor; then * sqrt(C), * gamma (bf16 ops)
  const float nrm = fmaxf(rbf(sqrtf(ss)), 1e-12f);
  unsigned short* yr = y + pix * C;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c0 = (i * 4 + q) * 8;
    u16x8 gw = *reinterpret_cast<const u16x8*>(gamma + c0);
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = rbf(v[i * 8 + e] / nrm);
      t = rbf(t * scale);
      t = rbf(t * bf2f(gw[e]));
      if (do_silu) t = t / (1.f + expf(-t));
      o[e] = f2bf(t);
    }
    *reinterpret_cast<u16x8*>(yr + c0) = o;
  }
}

template <int BK, int NT>
int launch_conv(const ConvArgs& a, hipStream_t s) {
  const int M = a.Ho * a.Wo;
  dim3 grid((unsigned)cdiv(M, kBM), (unsigned)cdiv(a.Cout, 32 * NT), (unsigned)a.Tout);
  hipLaunchKernelGGL((conv_igemm_kernel<BK, NT>), grid, dim3(256), 0, s, a);
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

// ---------------------------------------------------------------- AttentionBlock softmax
// P = softmax(S * scale) per row, fp32 scores in, bf16 probabilities out (the bf16 operand of the
// P.V GEMM). One 256-thread workgroup per row: pass 1 keeps a per-thread running (max, sum) over a
// strided slice of the row (float4 loads) and merges them across the block; pass 2 re-reads the row
// (L2-resident: a 14 080-column row is 56 KB) and writes exp2((s - max) c) / sum. HBM-bound.
__device__ __forceinline__ void ms_merge(float& m, float& l, float m2, float l2) {
  const float mn = fmaxf(m, m2);
  l = (m == -INFINITY ? 0.f : l * __builtin_amdgcn_exp2f(m - mn)) + (m2 == -INFINITY ? 0.f : l2 * __builtin_amdgcn_exp2f(m2 - mn));
  m = mn;
}

__global__ void __launch_bounds__(256) softmax_rows_kernel(const float* __restrict__ s, int64_t ld_s, int cols,
                                                           float c, unsigned short* __restrict__ p, int64_t ld_p,
                                                           int vec) {
  __shared__ float red_m[4], red_l[4];
  const float* row = s + (int64_t)blockIdx.x * ld_s;
  unsigned short* prow = p + (int64_t)blockIdx.x * ld_p;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n4 = vec ? cols >> 2 : 0;  // vec: rows 16-B (s) and 8-B (p) aligned
  float m = -INFINITY, l = 0.f;
  for (int i = tid; i < n4; i += 256) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(row + 4 * i);
#pragma unroll
    for (int e = 0; e < 4; ++e) ms_merge(m, l, v[e] * c, 1.f);
  }
  for (int i = 4 * n4 + tid; i < cols; i += 256) ms_merge(m, l, row[i] * c, 1.f);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const float m2 = __shfl_xor(m, off), l2 = __shfl_xor(l, off);
    ms_merge(m, l, m2, l2);
  }
  if (lane == 0) { red_m[wave] = m; red_l[wave] = l; }
  __syncthreads();
  m = red_m[0]; l = red_l[0];
#pragma unroll
  for (int w = 1; w < 4; ++w) ms_merge(m, l, red_m[w], red_l[w]);
  const float inv = 1.f / l;
  for (int i = tid; i < n4; i += 256) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(row + 4 * i);
    u16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = f2bf(__builtin_amdgcn_exp2f(v[e] * c - m) * inv);
    *reinterpret_cast<u16x4*>(prow + 4 * i) = o;
  }
  for (int i = 4 * n4 + tid; i < cols; i += 256) prow[i] = f2bf(__builtin_amdgcn_exp2f(row[i] * c - m) * inv);
}

}  // namespace

extern "C" int cp25_conv3d(const void* const* frames, int n_frames, const void* weight, const void* bias,
                           const void* residual, void* out, int Hin, int Win, int Cin, int Cout, int Tout, int KT,
                           int KH, int KW, int stride_t, int stride_hw, int pad_top, int pad_left, int pad_bottom,
                           int pad_right, int upsample, int out_split, hipStream_t stream) {
  if (n_frames < 1 || n_frames > kMaxFrames || !weight || !out || Tout < 1) return CP25_ERR_INVAL;
  if (Cin % 16 != 0 || Cin <= 0 || Cout <= 0) return CP25_ERR_DTYPE;
  if ((Tout - 1) * stride_t + KT > n_frames) return CP25_ERR_INVAL;
  if (out_split > 0 && (Cout != 2 * out_split || out_split % 4)) return CP25_ERR_INVAL;
  ConvArgs a;
  for (int i = 0; i < kMaxFrames; ++i) a.frames[i] = i < n_frames ? (const unsigned short*)frames[i] : nullptr;
  a.n_frames = n_frames;
  a.w = (const unsigned short*)weight;
  a.bias = (const unsigned short*)bias;
  a.residual = (const unsigned short*)residual;
  a.out = (unsigned short*)out;
  a.Hin = Hin; a.Win = Win; a.Cin = Cin; a.Cout = Cout; a.Tout = Tout;
  a.KT = KT; a.KH = KH; a.KW = KW;
  a.stride_t = stride_t; a.stride_hw = stride_hw; a.pad_top = pad_top; a.pad_left = pad_left;
  a.upsample = upsample;
  const int Hu = upsample ? 2 * Hin : Hin, Wu = upsample ? 2 * Win : Win;
  a.Ho = (Hu + pad_top + pad_bottom - KH) / stride_hw + 1;
  a.Wo = (Wu + pad_left + pad_right - KW) / stride_hw + 1;
  a.out_split = out_split;
  a.out_C = out_split > 0 ? out_split : Cout;
  if (a.Ho <= 0 || a.Wo <= 0) return CP25_ERR_INVAL;
  const int bk = (Cin % 64 == 0) ? 64 : (Cin % 32 == 0 ? 32 : 16);
  int nt;
  if (Cout <= 32) nt = 1;
  else if (Cout <= 64) nt = 2;
  else if (Cout % 96 == 0 && Cout <= 192) nt = 3;
  else nt = 4;
#define CONV_CASE(BK_, NT_) if (bk == BK_ && nt == NT_) return launch_conv<BK_, NT_>(a, stream);
  CONV_CASE(16, 1) CONV_CASE(16, 2) CONV_CASE(16, 3) CONV_CASE(16, 4)
  CONV_CASE(32, 1) CONV_CASE(32, 2) CONV_CASE(32, 3) CONV_CASE(32, 4)
  CONV_CASE(64, 1) CONV_CASE(64, 2) CONV_CASE(64, 3) CONV_CASE(64, 4)
#undef CONV_CASE
  return CP25_ERR_DTYPE;
}

extern "C" int cp25_softmax_rows(const float* s, int64_t rows, int cols, int64_t ld_s, float scale, void* p,
                                 int64_t ld_p, hipStream_t stream) {
  if (!s || !p || rows <= 0 || cols <= 0 || ld_s < cols || ld_p < cols || !(scale > 0.f)) return CP25_ERR_INVAL;
  if (((uintptr_t)s & 3) || ((uintptr_t)p & 1) || rows > 0x7fffffff) return CP25_ERR_INVAL;
  const int vec = !((uintptr_t)s & 15) && !((uintptr_t)p & 7) && !(ld_s & 3) && !(ld_p & 3);
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)rows), dim3(256), 0, stream, s, ld_s, cols,
                     scale * 1.4426950408889634f, (unsigned short*)p, ld_p, vec);
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

extern "C" int cp25_rms_norm_silu(const void* x, const void* gamma, void* y, int64_t n_pix, int C, int do_silu,
                                  hipStream_t stream) {
  if (!x || !gamma || !y || n_pix <= 0 || C % 32 != 0) return CP25_ERR_INVAL;
  const float scale = (float)sqrt((double)C);  // python float dim**0.5, rounded to fp32 by the bf16 mul
  const dim3 grid((unsigned)cdiv(n_pix, 64));
#define RNS(V) hipLaunchKernelGGL(rms_norm_silu_kernel<V>, grid, dim3(256), 0, stream, (const unsigned short*)x, \
                                  (const unsigned short*)gamma, (unsigned short*)y, n_pix, scale, do_silu)
  switch (C / 32) {
    case 1: RNS(1); break;
    case 2: RNS(2); break;
    case 3: RNS(3); break;
    case 6: RNS(6); break;
    case 12: RNS(12); break;
    default: return CP25_ERR_DTYPE;
  }
#undef RNS
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}
