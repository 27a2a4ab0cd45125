// Flash-attention forward for the DiT self- and cross-attention (gfx950, bf16 in/out, head dim 128).
//
// Replaces the reference's attention op: cosmos_predict2/_src/predict2/networks/attention.py:90-181
// (q/k/v recast to bf16, softmax(QK^T / sqrt(D)) V, no mask, no dropout, non-causal), which the DiT
// calls through MinimalA2AAttnOp (networks/a2a_cp.py:208-219) on [B, S, H, D] tensors.
//
// Design (MI355X-first, see DESIGN.md "attn_fwd"):
//   * one workgroup = 8 waves = 256 query rows of one (batch, head); every wave owns 32 query rows;
//   * K/V stream through LDS in 64-key tiles, double buffered, register-staged (issue global loads
//     before the MFMA work on the current tile, write LDS after it), ONE barrier per tile;
//   * "swapped" products so the softmax is lane-local: S^T = K Q^T (v_mfma_f32_32x32x16_bf16, the
//     query on the lane), then O^T = V^T P^T, whose B operand is the S accumulator converted to bf16
//     with no lane movement, and whose A operand (V^T) comes from ds_read_b64_tr_b16 (hardware
//     transposed LDS read) of the row-major V tile;
//   * padded LDS rows (K 272 B, V 320 B) keep both the ds_read_b128 row reads of K and the transposed
//     reads of V bank-conflict-free with every address a per-lane base + immediate; the tile loop is
//     unrolled over the two LDS buffers so no address arithmetic remains in it;
//   * the O rescale of the online softmax is skipped (exactly) when no row max of the wave grew;
//   * grid remapped so the workgroups of one XCD share a (batch, head): their K/V stream hits in
//     that XCD's L2 instead of HBM.
// Numerics: scores and the running max/sum are fp32, P is rounded to bf16 before P.V (as every
// flash-attention kernel the reference dispatches to does), O is accumulated in fp32, normalised
// and rounded once to bf16.
#include "cp25_common.h"

#include <type_traits>

namespace {

constexpr int kD = 128;        // head dim
constexpr int kWaves = 8;      // waves per workgroup
constexpr int kQRows = 32;     // query rows per wave
constexpr int kQBlk = kWaves * kQRows;  // 256 query rows per workgroup
constexpr int kKBlk = 64;      // keys per tile
constexpr int kThreads = kWaves * 64;
// LDS layout (bytes): [V0 | V1 | K0 | K1]. Padded rows instead of an XOR swizzle so every LDS read
// is one per-lane base VGPR + a compile-time immediate (no per-tile address arithmetic):
//   K rows 272 B (256 + 16): the 16 rows a ds_read_b128 lane group reads at one column land on 16
//     distinct 16-B bank slots;
//   V rows 320 B (256 + 64): the 4 rows x 64 B a half-wave of ds_read_b64_tr_b16 reads land on the
//     4 distinct 64-B quarters of the 256-B bank row.
constexpr int kKStride = 272;
constexpr int kVStride = 320;
constexpr int kVBuf = kKBlk * kVStride;  // 20480
constexpr int kKBuf = kKBlk * kKStride;  // 17408
constexpr int kV0 = 0, kV1 = kVBuf, kK0 = 2 * kVBuf, kK1 = 2 * kVBuf + kKBuf;
constexpr int kLdsBytes = 2 * kVBuf + 2 * kKBuf;  // 75776

typedef __attribute__((address_space(3))) s16x4* lds_s16x4_ptr;

__device__ __forceinline__ bf16x8 tr_read_pair(const char* pa, const char* pb) {
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_ptr)pa);
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_ptr)pb);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, r);
}

__device__ __forceinline__ float wave_swap_max(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float wave_swap_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

struct AttnArgs {
  const unsigned short* q; const unsigned short* k; const unsigned short* v; unsigned short* o;
  int64_t q_sb, q_sl, q_sh;
  int64_t k_sb, k_sl, k_sh;
  int64_t v_sb, v_sl, v_sh;
  int64_t o_sb, o_sl, o_sh;
  int B, H, Lq, Lk;
  int nqb;          // query blocks per (b, h)
  float scale_log2; // softmax scale * log2(e)
};

template <int kKind>  // 0: self-attention, 1: cross-attention (separate symbols in profiles)
__global__ void __launch_bounds__(kThreads, 2) attn_fwd_d128(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];

  const int nwg = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int bh = tile / a.nqb, qb = tile % a.nqb;
  const int b = bh / a.H, h = bh % a.H;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int l31 = lane & 31;
  const int hl = lane >> 5;  // lane half

  const unsigned short* qp = a.q + b * a.q_sb + h * a.q_sh;
  const unsigned short* kp = a.k + b * a.k_sb + h * a.k_sh;
  const unsigned short* vp = a.v + b * a.v_sb + h * a.v_sh;

  // ---- Q fragments (B operand of S^T = K Q^T): Q[q][16s + 8hl .. +7], s = 0..7 ----
  const int q_row = qb * kQBlk + wave * kQRows + l31;
  const int q_row_c = q_row < a.Lq ? q_row : a.Lq - 1;
  bf16x8 qf[8];
  {
    const unsigned short* src = qp + (int64_t)q_row_c * a.q_sl + 8 * hl;
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(src + 16 * s);
  }

  f32x16 o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m_run = -1e30f;
  float l_run = 0.f;

  const int ntiles = (a.Lk + kKBlk - 1) / kKBlk;

  // staging: each thread owns 2 K chunks and 2 V chunks (16 B each) of a 64x128 tile
  const int srow0 = tid >> 4, sch = tid & 15;  // chunk i: row srow0 + 32 i
  u32x4 stK[2], stV[2];
  // branch-free staging loads: rows past the end are clamped to the last key (finite data; their
  // scores are masked to -inf and their P is 0), tiles past the end re-load the last tile (unused)
  auto load_rows = [&](const unsigned short* base, int64_t sl, int t, u32x4 (&dst)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int key = min(t * kKBlk + srow0 + 32 * i, a.Lk - 1);
      dst[i] = *reinterpret_cast<const u32x4*>(base + (int64_t)key * sl + sch * 8);
    }
  };
  char* const k_wr = smem + srow0 * kKStride + sch * 16;
  char* const v_wr = smem + srow0 * kVStride + sch * 16;
  auto write_k = [&](auto BUF) {
    constexpr int kb = decltype(BUF)::value ? kK1 : kK0;
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4*>(k_wr + kb + 32 * i * kKStride) = stK[i];
  };
  auto write_v = [&](auto BUF) {
    constexpr int vb = decltype(BUF)::value ? kV1 : kV0;
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4*>(v_wr + vb + 32 * i * kVStride) = stV[i];
  };

  // per-lane LDS read bases (everything else is an immediate offset)
  const char* const k_rd = smem + l31 * kKStride + 16 * hl;  // + kt*32 rows + 32 s bytes
  const int grp = lane >> 4, gi = lane & 15;
  const int tq = gi >> 2, tp = gi & 3;
  const char* const v_rd = smem + (4 * (grp >> 1) + tq) * kVStride + 32 * (grp & 1) + 8 * tp;  // + rows, + 64 db

  // ragged last tile: its accumulator starts at -inf on keys >= Lk (masking folded into S's C operand)
  const bool ragged = (a.Lk % kKBlk) != 0;

  // S^T(tile in K buffer) = K Q^T. init: zeros, or -inf on keys >= Lk for the ragged last tile
  // (masking folded into the MFMA's C operand)
  auto qk_init = [&](int t, f32x16 (&S)[2]) {
    if (ragged && t == ntiles - 1) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = t * kKBlk + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
          S[kt][r] = key < a.Lk ? 0.f : -INFINITY;
        }
    } else {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) S[kt][r] = 0.f;
    }
  };
  auto qk_mma = [&](auto BUF, f32x16 (&S)[2]) {
    constexpr int kb = decltype(BUF)::value ? kK1 : kK0;
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(k_rd + kb + kt * 32 * kKStride + 32 * s);
        S[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], S[kt], 0, 0, 0);
      }
  };
  // online softmax, part 1: running max and (only if some row max grew: exact skip) the O rescale
  auto sm_max = [&](f32x16 (&S)[2]) {
    float mx = fmaxf(S[0][0], S[1][0]);
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, fmaxf(S[0][r], S[1][r]));
    mx = wave_swap_max(mx);
    const float m_new = fmaxf(m_run, mx * a.scale_log2);
    if (__any(m_new > m_run)) {
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      l_run *= alpha;
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[d][r] *= alpha;
      m_run = m_new;
    }
  };
  // part 2: P = exp2(S c - m) -> bf16 (lane-local B operand), row sum, O^T += V^T P^T
  auto sm_pv = [&](auto BUF, f32x16 (&S)[2]) {
    constexpr int vb = decltype(BUF)::value ? kV1 : kV0;
    bf16x8 pb[4];
    float psum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float p = __builtin_amdgcn_exp2f(fmaf(S[kt][8 * sp + j], a.scale_log2, -m_run));
          psum += p;
          v[j] = static_cast<__bf16>(p);
        }
        pb[2 * kt + sp] = v;
      }
    l_run += psum;
#pragma unroll
    for (int Sx = 0; Sx < 4; ++Sx)
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const char* pa = v_rd + vb + (16 * Sx) * kVStride + 64 * db;
        const bf16x8 vf = tr_read_pair(pa, pa + 8 * kVStride);
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pb[Sx], o[db], 0, 0, 0);
      }
  };

  // Software pipeline, K one tile ahead of V. Iteration t: QK^T of tile t+1 (K buffer (t+1)&1) is
  // issued before the softmax + PV of tile t (V buffer t&1), so the matrix pipe stays busy while
  // the VALU finishes the softmax. Registers prefetch K(t+2), V(t+1); after the compute they go to
  // K buffer t&1 (K(t) was last read in iteration t-1) and V buffer (t+1)&1 (V(t-1), iteration t-1).
  typedef std::integral_constant<int, 0> B0;
  typedef std::integral_constant<int, 1> B1;
  f32x16 SA[2], SB[2];
  load_rows(kp, a.k_sl, 0, stK);
  load_rows(vp, a.v_sl, 0, stV);
  write_k(B0{});
  write_v(B0{});
  load_rows(kp, a.k_sl, 1, stK);
  write_k(B1{});
  __syncthreads();
  qk_init(0, SA);
  qk_mma(B0{}, SA);
  __syncthreads();  // K buffer 0 is rewritten in iteration 0
  for (int t = 0; t < ntiles; t += 2) {
    // -- even tile t: scores SA, K(t+1) in buffer 1, V(t) in buffer 0
    load_rows(kp, a.k_sl, t + 2, stK);
    load_rows(vp, a.v_sl, t + 1, stV);
    qk_init(t + 1, SB);
    sm_max(SA);
    qk_mma(B1{}, SB);
    sm_pv(B0{}, SA);
    write_k(B0{});
    write_v(B1{});
    __syncthreads();
    if (t + 1 >= ntiles) break;
    // -- odd tile t+1: scores SB, K(t+2) in buffer 0, V(t+1) in buffer 1
    load_rows(kp, a.k_sl, t + 3, stK);
    load_rows(vp, a.v_sl, t + 2, stV);
    qk_init(t + 2, SA);
    sm_max(SB);
    qk_mma(B0{}, SA);
    sm_pv(B1{}, SB);
    write_k(B1{});
    write_v(B0{});
    __syncthreads();
  }

  // ---- epilogue: O = O^T / l, bf16, row q, d = 32db + 8g + 4hl + (0..3) ----
  const float l_tot = wave_swap_sum(l_run);
  const float inv = 1.f / l_tot;
  if (q_row < a.Lq) {
    unsigned short* op = a.o + b * a.o_sb + h * a.o_sh + (int64_t)q_row * a.o_sl;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = f2bf(o[db][4 * g + e] * inv);
        *reinterpret_cast<u16x4*>(op + 32 * db + 8 * g + 4 * hl) = w;
      }
  }
}

}  // namespace

extern "C" int cp25_attn_fwd(const void* q, const void* k, const void* v, void* o, int B, int H, int Lq,
                             int Lk, int D, const int64_t* q_strides, const int64_t* k_strides,
                             const int64_t* v_strides, const int64_t* o_strides, float softmax_scale,
                             hipStream_t stream) {
  if (D != kD) return CP25_ERR_DTYPE;
  if (B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0) return CP25_ERR_INVAL;
  if (!q || !k || !v || !o) return CP25_ERR_INVAL;
  // rows must be 16-byte aligned for the vector loads / stores; head dim contiguous
  const int64_t* ss[4] = {q_strides, k_strides, v_strides, o_strides};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 3; ++j)
      if (ss[i][j] % 8 != 0) return CP25_ERR_INVAL;
  if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) & 15) return CP25_ERR_INVAL;
  AttnArgs a;
  a.q = (const unsigned short*)q; a.k = (const unsigned short*)k; a.v = (const unsigned short*)v;
  a.o = (unsigned short*)o;
  a.q_sb = q_strides[0]; a.q_sl = q_strides[1]; a.q_sh = q_strides[2];
  a.k_sb = k_strides[0]; a.k_sl = k_strides[1]; a.k_sh = k_strides[2];
  a.v_sb = v_strides[0]; a.v_sl = v_strides[1]; a.v_sh = v_strides[2];
  a.o_sb = o_strides[0]; a.o_sl = o_strides[1]; a.o_sh = o_strides[2];
  a.B = B; a.H = H; a.Lq = Lq; a.Lk = Lk;
  a.nqb = (int)cdiv(Lq, kQBlk);
  a.scale_log2 = softmax_scale * 1.4426950408889634f;
  const int64_t nwg = (int64_t)a.nqb * B * H;
  if (nwg > 0x7fffffff) return CP25_ERR_INVAL;
  if (Lk <= 4096)
    hipLaunchKernelGGL(attn_fwd_d128<1>, dim3((unsigned)nwg), dim3(kThreads), 0, stream, a);
  else
    hipLaunchKernelGGL(attn_fwd_d128<0>, dim3((unsigned)nwg), dim3(kThreads), 0, stream, a);
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}
