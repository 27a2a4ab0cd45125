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

#include <cstdlib>
#include <cstring>
#include <type_traits>

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


// ---------------------------------------------------------------- 3x3 stride-1 conv with an LDS halo tile
// The 3x3(x3) convs of the ResidualBlocks and the upsample Resample convs (pad 1 left / right; any top / bottom
// pad, so the row bands of the banded decode take the same kernel and the same summation order). A workgroup
// (NW = 8 waves, two per SIMD, so one wave's LDS / DMA waits are covered by its partner's MFMAs; or NW = 4, one per
// SIMD) owns a TH x TW output tile (512 pixels: each wave 16 / NW fragments of 32 pixels of a row)
// x BN = 32 NT output channels, and walks the K dimension in stages of (temporal tap kt, 16 input channels):
//   * per stage the (TH + 2) x (TW + 2) input halo (16 channels, 32 B per pixel) and the 9 x BN weight rows of
//     the stage land in LDS by LDS-DMA (global_load_lds_dwordx4, 32 pixels / couts per wave instruction;
//     padding, rows past Ho and causal zero frames read a zero page), through a 3-deep LDS ring: stage s + 2's
//     DMA is in flight while stage s is multiplied (counted vmcnt, raw barriers);
//   * the 9 spatial taps then read shifted windows of the same halo: each input pixel is fetched from global
//     memory once per (kt, channel chunk) instead of 9 times, and every LDS read is a contiguous 1-KiB wave read
//     ([pixel][16 ch] and [tap][cout][16 ch] images: conflict-free without a swizzle);
//   * per stage and wave 9 x 4 x NT MFMAs (v_mfma_f32_32x32x16_bf16) against 9 (4 + NT) fragment reads, so the
//     LDS read rate stays under the one 1-KiB read per MFMA a SIMD can be fed (the per-tap kernel above reads
//     1.3 per MFMA and is LDS-bound).
// Same accumulation order over k = (kt, kh, kw, ci) per output as conv_igemm_kernel except the order of the
// channel chunks within a tap, so results match it to fp32 rounding.
__device__ __attribute__((aligned(16))) unsigned int g_zero_page[64];

// compile-time loop: f(integral_constant<int, I>) for I = 0 .. N-1, in order
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}  // 256 B of zeros (static storage)

template <int NT, int TW, int NW>
__global__ void __launch_bounds__(64 * NW, 1) conv3x3_halo_kernel(ConvArgs a) {
  constexpr int BN = 32 * NT;
  constexpr int FPW = 16 / NW;                     // 32-pixel fragments per wave (16 per 512-pixel tile)
  constexpr int TH = 512 / TW;
  constexpr int HWD = TW + 2, HHT = TH + 2;
  constexpr int NHP = HWD * HHT;                   // halo pixels
  constexpr int W_INS = 9 * NT;                    // wave instructions (32 couts x 32 B) per stage
  // wave instructions (32 pixels x 32 B) for the halo, padded so every wave issues the same count per stage
  // (the padding instructions copy the zero page into LDS past the halo): the counted vmcnt below needs it
  constexpr int HALO_INS = ((NHP + 31) / 32 + W_INS + 3) / 4 * 4 - W_INS;
  constexpr int HALO_BYTES = HALO_INS * 1024;
  constexpr int STAGE = HALO_BYTES + W_INS * 1024;
  constexpr int N_INS = HALO_INS + W_INS;
  constexpr int INS_PER_WAVE = (N_INS + NW - 1) / NW;  // the most any wave issues per stage (waves >= N_INS % NW
                                                       // issue one fewer when NW does not divide N_INS)
  constexpr int FPR = TW / 32;                     // fragments per tile row
  constexpr int NBUF = 3;                          // LDS ring: stage s + 2's DMA in flight while s is multiplied
  static_assert(N_INS % 4 == 0 && NBUF * STAGE <= 160 * 1024 && (NW == 4 || NW == 8), "halo conv LDS");
  __shared__ __attribute__((aligned(16))) char smem[NBUF * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l31 = lane & 31, hl = lane >> 5;
  // grid.x = (spatial tile, output frame) with the frame fastest, XCD-remapped: the Tout workgroups of one spatial
  // tile run together on one XCD and share their input halos (a frame feeds KT output frames) through its L2
  const int tiles_w = a.Wo / TW;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int to = lin % a.Tout, tile = lin / a.Tout;
  const int th0 = (tile / tiles_w) * TH, tw0 = (tile % tiles_w) * TW;
  const int n0 = blockIdx.y * BN;
  const int kc = a.Cin / 16;
  const int nst = a.KT * kc;

  // ---- this lane's DMA sources (stage independent part): instruction i = wave + NW u
  //   halo: pixel offset (hi * Win + wi) * Cin + 8 half, or -1 (zero page)
  //   weights: ((cout * KT) * 9 + tap) * Cin + 8 half, or -1; + kt * 9 * Cin + c16 * 16 per stage
  // lane l of a DMA instruction moves 16 B (8 channels) of pixel / cout l % 32, channel half l / 32: the LDS images
  // are [32-pixel block][half][32][16 B] and [tap][cout block][half][32][16 B], so a fragment read (32 pixels or
  // couts x one half per 32 lanes) is 512 contiguous bytes: bank-conflict-free
  const int half = lane >> 5, sub = lane & 31;
  int src_off[INS_PER_WAVE];
#pragma unroll
  for (int u = 0; u < INS_PER_WAVE; ++u) {
    const int i = wave + NW * u;  // (i >= N_INS: this wave has one instruction fewer; never issued)
    int off = -1;  // -1: the zero page
    if (i < HALO_INS) {
      const int h = i * 32 + sub;
      if (h < NHP) {
        const int hr = h / HWD, hc = h % HWD;
        const int hu = th0 - a.pad_top + hr, wu = tw0 - a.pad_left + hc;  // (upsampled) input coordinates
        const int Hs = a.upsample ? 2 * a.Hin : a.Hin, Ws = a.upsample ? 2 * a.Win : a.Win;
        if (hu >= 0 && hu < Hs && wu >= 0 && wu < Ws) {
          const int hi = a.upsample ? hu >> 1 : hu, wi = a.upsample ? wu >> 1 : wu;
          off = (hi * a.Win + wi) * a.Cin + 8 * half;
        }
      }
    } else if (i < N_INS) {
      const int wi_ = i - HALO_INS;
      const int tap = wi_ / NT, cb = wi_ % NT;
      const int co = n0 + cb * 32 + sub;
      if (co < a.Cout) off = (co * a.KT * 9 + tap) * a.Cin + 8 * half;
    }
    src_off[u] = off;
  }
  const unsigned short* zero = reinterpret_cast<const unsigned short*>(g_zero_page);

  // the (up to 3) input frames of this output frame, read from the kernel arguments once: a dynamically indexed
  // argument load inside the loop is an SMEM access, and with one in flight the compiler's LDS waits degrade to
  // lgkmcnt(0)
  const unsigned short* frk[3];
#pragma unroll
  for (int kt = 0; kt < 3; ++kt) {
    const int fi = to * a.stride_t + kt;
    frk[kt] = (kt < a.KT && fi < a.n_frames) ? a.frames[fi] : nullptr;
  }
  auto issue = [&](int st, int buf) __attribute__((always_inline)) {
    const int kt = st / kc, c16 = (st % kc) * 16;
    const unsigned short* fr = kt == 0 ? frk[0] : (kt == 1 ? frk[1] : frk[2]);
    const unsigned short* wst = a.w + kt * 9 * a.Cin + c16;
    char* base = smem + buf * STAGE;
#pragma unroll
    for (int u = 0; u < INS_PER_WAVE; ++u) {
      const int i = wave + NW * u;
      if (N_INS % NW != 0 && i >= N_INS) break;  // wave-uniform
      {
        const unsigned short* src;
        char* dst;
        if (i < HALO_INS) {
          src = (fr != nullptr && src_off[u] >= 0) ? fr + src_off[u] + c16 : zero;
          dst = base + i * 1024;
        } else {
          src = src_off[u] >= 0 ? wst + src_off[u] : zero;
          dst = base + HALO_BYTES + (i - HALO_INS) * 1024;
        }
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      }
    }
  };

  // counted wait for the stage after next: this wave's DMA instructions of one stage stay in flight
  const bool short_wave = N_INS % NW != 0 && wave >= N_INS % NW;
  auto wait_stage_dma = [&](auto LGK) __attribute__((always_inline)) {
    if (short_wave) {
      if constexpr (decltype(LGK)::value)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(INS_PER_WAVE - 1) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(INS_PER_WAVE - 1) : "memory");
    } else {
      if constexpr (decltype(LGK)::value)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(INS_PER_WAVE) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(INS_PER_WAVE) : "memory");
    }
  };

  f32x16 acc[FPW][NT];
#pragma unroll
  for (int f = 0; f < FPW; ++f)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[f][j][r] = 0.f;

  // fragment f of this wave: tile row (FPW wave + f) / FPR, columns ((FPW wave + f) % FPR) 32 + [0, 32); its halo
  // pixel for tap (kh, kw) is h = h0[f] + kh HWD + kw, at byte (h / 32) 1024 + hl 512 + (h % 32) 16
  int h0[FPW];
#pragma unroll
  for (int f = 0; f < FPW; ++f) {
    const int q = wave * FPW + f;
    h0[f] = (q / FPR) * HWD + (q % FPR) * 32 + l31;
  }
  const int b_base = HALO_BYTES + hl * 512 + l31 * 16;
  static_assert(NT == 3, "the counted LDS waits below assume 3 + FPW fragment reads per tap");
  typedef __attribute__((address_space(3))) const char* lds_cptr;
  const unsigned smem_lds = (unsigned)(uintptr_t)(lds_cptr)smem;

  // Pipeline: stage s + 2 is queued at the top of stage s (into the buffer stage s - 1 used: every wave passed
  // the barrier after it); the counted wait at the bottom retires stage s + 1 only (raw barrier: a
  // __syncthreads() fence would drain the DMA queue).
  issue(0, 0);
  if (nst > 1) {
    issue(1, 1);
    wait_stage_dma(std::false_type{});
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  int buf = 0;
  for (int st = 0; st < nst; ++st) {
    if (st + 2 < nst) issue(st + 2, buf == 0 ? 2 : buf - 1);
    // fragments of tap t + 1 are read (inline asm, 3 B + FPW A reads) while tap t's 3 FPW MFMAs issue, behind a
    // counted lgkmcnt(3 + FPW) tied to tap t's registers (the compiler's own waits here were lgkmcnt(0): a full LDS
    // latency every other tap)
    const unsigned sbase = smem_lds + buf * STAGE;
    const unsigned b_addr = sbase + b_base;
    bf16x8 xa[2][FPW], wb[2][NT];
    auto load_tap = [&](auto TC, bf16x8(&xs)[FPW], bf16x8(&ws)[NT]) __attribute__((always_inline)) {
      constexpr int tap = decltype(TC)::value, kh = tap / 3, kw = tap % 3;
#pragma unroll
      for (int j = 0; j < NT; ++j)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ws[j]) : "v"(b_addr), "i"((tap * NT + j) * 1024));
#pragma unroll
      for (int f = 0; f < FPW; ++f) {
        const int h = h0[f] + kh * HWD + kw;
        const unsigned ad = sbase + (h >> 5) * 1024 + hl * 512 + (h & 31) * 16;
        asm volatile("ds_read_b128 %0, %1" : "=v"(xs[f]) : "v"(ad));
      }
    };
    load_tap(std::integral_constant<int, 0>{}, xa[0], wb[0]);
    static_for<9>([&](auto TC) __attribute__((always_inline)) {
      constexpr int tap = decltype(TC)::value, cur = tap & 1;
      if constexpr (tap + 1 < 9) {
        load_tap(std::integral_constant<int, tap + 1>{}, xa[cur ^ 1], wb[cur ^ 1]);
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(NT + FPW));
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)");
      }
      // tap t's operands are ready only after the wait: pin them behind it
#pragma unroll
      for (int j = 0; j < NT; ++j) asm volatile("" : "+v"(wb[cur][j]));
#pragma unroll
      for (int f = 0; f < FPW; ++f) asm volatile("" : "+v"(xa[cur][f]));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int f = 0; f < FPW; ++f)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[f][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wb[cur][j], xa[cur][f], acc[f][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    });
    if (st + 2 < nst)
      wait_stage_dma(std::true_type{});
    else
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    buf = buf == NBUF - 1 ? 0 : buf + 1;
  }

  // ---- epilogue through LDS: bf16(acc + bias) -> [512 px][BN] image (row stride BN * 2 + 8 B: the 8-B writes of
  // a fragment's 32 pixels hit distinct banks), then 16-B chunks of whole pixel rows to global, + residual
  constexpr int OST = BN * 2 + 8;
  static_assert(512 * OST <= NBUF * STAGE, "halo conv epilogue staging");
#pragma unroll
  for (int f = 0; f < FPW; ++f) {
    const int px = (wave * FPW + f) * 32 + l31;  // tile pixel (fragment-major = row-major within the tile)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int cl = j * 32 + 8 * g + 4 * hl;
        u16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = acc[f][j][4 * g + e];
          if (a.bias != nullptr && n0 + cl + e < a.Cout) x += bf2f(a.bias[n0 + cl + e]);
          w[e] = f2bf(x);
        }
        *reinterpret_cast<u16x4*>(smem + px * OST + cl * 2) = w;
      }
  }
  __syncthreads();
  const int M = a.Ho * a.Wo;
  constexpr int CPP = BN / 8;  // 16-B chunks per pixel
  const bool vec_ok = (a.Cout % 8) == 0 && n0 + BN <= a.Cout;
  for (int idx = tid; idx < 512 * CPP; idx += 64 * NW) {
    const int px = idx / CPP, c = idx % CPP;
    const int q = px >> 5;
    const int ho = th0 + q / FPR, wo = tw0 + (q % FPR) * 32 + (px & 31);
    if (ho >= a.Ho) continue;
    const int64_t o = ((int64_t)to * M + (int64_t)ho * a.Wo + wo) * a.Cout + n0 + c * 8;
    const u16x8 cv = *reinterpret_cast<const u16x8*>(smem + px * OST + c * 16);
    if (vec_ok) {
      u16x8 w = cv;
      if (a.residual != nullptr) {
        const u16x8 r = *reinterpret_cast<const u16x8*>(a.residual + o);
#pragma unroll
        for (int e = 0; e < 8; ++e) w[e] = f2bf(bf2f(cv[e]) + bf2f(r[e]));
      }
      *reinterpret_cast<u16x8*>(a.out + o) = w;
    } else {
      for (int e = 0; e < 8; ++e) {
        if (n0 + c * 8 + e >= a.Cout) break;
        float v = bf2f(cv[e]);
        if (a.residual != nullptr) v = rbf(v + bf2f(a.residual[o + e]));
        a.out[o + e] = f2bf(v);
      }
    }
  }
}

template <int NT, int TW, int NW>
int launch_conv_halo(const ConvArgs& a, hipStream_t s) {
  constexpr int TH = 512 / TW;
  dim3 grid((unsigned)(cdiv(a.Ho, TH) * (a.Wo / TW) * a.Tout), (unsigned)cdiv(a.Cout, 32 * NT), 1u);
  hipLaunchKernelGGL((conv3x3_halo_kernel<NT, TW, NW>), grid, dim3(64 * NW), 0, s, a);
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

// conv kernel selection, set once at library load from CP25_CONV_KERNEL ("tap": the per-tap kernel only) and
// changed only through cp25_conv3d_select (never read from the environment per launch)
static int g_conv_select = [] {
  const char* e = std::getenv("CP25_CONV_KERNEL");
  return (e && !std::strcmp(e, "tap")) ? 1 : 0;
}();

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
  // 3x3 stride-1 pad-1 convs: the halo kernel (cp25_conv3d_select(1) selects the per-tap kernel, A/B and tests)
  // (any top / bottom pad: the banded decode passes haloed bands with pads 0 or -1 there)
  const bool halo_ok = KH == 3 && KW == 3 && stride_hw == 1 && out_split == 0 && pad_left == 1 && pad_right == 1 &&
                       Cout >= 64 && KT <= 3 && a.Wo % 32 == 0 &&
                       (int64_t)Hin * Win * Cin < (1LL << 31) && (int64_t)Cout * KT * 9 * Cin < (1LL << 31) &&
                       g_conv_select != 1;
  if (halo_ok) {
    // BN = 96 for every Cout (96 / 192 / 384 in the decoder): with BN = 128 the 256 accumulators spill
    // 8 waves (two per SIMD, 2 fragments each; the default): 8-16 % faster than 4 waves (one per SIMD, 4
    // fragments each, cp25_conv3d_select(2)) at the decoder's shapes, bit-identical (profiles/r3/conv/)
    // 512-pixel tiles of 16 rows x 32 columns: an 18 x 34 halo (1.20 x the tile) instead of 6 x 130 for 4 x 128 (1.52 x):
    // 4-6 % faster at the 96- and 192-channel shapes, equal at 384 (profiles/r3/conv/tile_width_ab.log); the sums
    // per output are the same MFMA chains whatever the tile shape, so the results are bit-identical
    if (g_conv_select == 2) return launch_conv_halo<3, 32, 4>(a, stream);
    return launch_conv_halo<3, 32, 8>(a, stream);
  }
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

extern "C" int cp25_conv3d_select(int mode) {
  if (mode < 0 || mode > 2) return CP25_ERR_INVAL;
  const int prev = g_conv_select;
  g_conv_select = mode;
  return prev;
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
