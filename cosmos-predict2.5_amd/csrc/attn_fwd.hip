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
//   * one XOR swizzle of the 256-byte LDS rows serves both the ds_read_b128 row reads of K and the
//     transposed reads of V without bank conflicts;
//   * grid remapped so the workgroups of one XCD share a (batch, head): their K/V stream hits in
//     that XCD's L2 instead of HBM.
// Numerics: scores and the running max/sum are fp32, P is rounded to bf16 before P.V (as every
// flash-attention kernel the reference dispatches to does), O is accumulated in fp32, normalised
// and rounded once to bf16.
#include "cp25_common.h"

namespace {

constexpr int kD = 128;        // head dim
constexpr int kWaves = 8;      // waves per workgroup
constexpr int kQRows = 32;     // query rows per wave
constexpr int kQBlk = kWaves * kQRows;  // 256 query rows per workgroup
constexpr int kKBlk = 64;      // keys per tile
constexpr int kThreads = kWaves * 64;
constexpr int kTileBytes = kKBlk * kD * 2;  // 16 KiB
// LDS: [buf][K|V][64 rows][256 B]
constexpr int kLdsBytes = 2 * 2 * kTileBytes;

// 16-byte chunk swizzle inside a 256-byte row (cdna_hip_programming.md T10 image (b)).
__device__ __forceinline__ int swz(int row, int ch) { return ch ^ (((row & 3) << 2) | ((row >> 2) & 3)); }
__device__ __forceinline__ int lds_off(int row, int ch) { return row * 256 + 16 * swz(row, ch); }

typedef __attribute__((address_space(3))) s16x4* lds_s16x4_ptr;

__device__ __forceinline__ bf16x8 tr_read_pair(const char* smem, int off_a, int off_b) {
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_ptr)(smem + off_a));
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_ptr)(smem + off_b));
  s16x4 lo = a, hi = b;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
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
  u32x4 stK[2], stV[2];
  auto stage_load = [&](int t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + kThreads * i;
      const int row = c >> 4, ch = c & 15;
      const int key = t * kKBlk + row;
      if (key < a.Lk) {
        stK[i] = *reinterpret_cast<const u32x4*>(kp + (int64_t)key * a.k_sl + ch * 8);
        stV[i] = *reinterpret_cast<const u32x4*>(vp + (int64_t)key * a.v_sl + ch * 8);
      } else {
        stK[i] = u32x4{0u, 0u, 0u, 0u};
        stV[i] = u32x4{0u, 0u, 0u, 0u};
      }
    }
  };
  auto stage_write = [&](int buf) {
    char* kb = smem + buf * 2 * kTileBytes;
    char* vb = kb + kTileBytes;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + kThreads * i;
      const int row = c >> 4, ch = c & 15;
      *reinterpret_cast<u32x4*>(kb + lds_off(row, ch)) = stK[i];
      *reinterpret_cast<u32x4*>(vb + lds_off(row, ch)) = stV[i];
    }
  };

  stage_load(0);
  stage_write(0);
  __syncthreads();

  // per-lane constant pieces of the V transposed-read address
  const int grp = lane >> 4;        // 16-lane group
  const int gi = lane & 15;         // index inside the group: 4q + p
  const int tq = gi >> 2, tp = gi & 3;
  const int trow_base = 4 * (grp >> 1) + tq;          // + 16*S (+8 for the second read)
  const int tch_base = 2 * (grp & 1) + (tp >> 1);     // + 4*db
  const int tbyte = 8 * (tp & 1);

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) stage_load(t + 1);

    const char* kb = smem + buf * 2 * kTileBytes;
    const char* vb = kb + kTileBytes;

    // ---- S^T = K Q^T : two 32-key halves ----
    f32x16 sacc[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[kt][r] = 0.f;
      const int krow = kt * 32 + l31;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        bf16x8 kf = *reinterpret_cast<const bf16x8*>(kb + lds_off(krow, 2 * s + hl));
        sacc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc[kt], 0, 0, 0);
      }
    }

    // ---- mask the ragged last tile ----
    if ((t + 1) * kKBlk > a.Lk) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = t * kKBlk + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (key >= a.Lk) sacc[kt][r] = -INFINITY;
        }
    }

    // ---- online softmax (lane-local: this lane + lane^32 hold one query row) ----
    float mx = sacc[0][0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sacc[0][r]);
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[1][r]);
    mx = wave_swap_max(mx);
    const float m_new = fmaxf(m_run, mx * a.scale_log2);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    m_run = m_new;

    bf16x8 pb[4];
    float psum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float p = __builtin_amdgcn_exp2f(fmaf(sacc[kt][8 * sp + j], a.scale_log2, -m_new));
          psum += p;
          v[j] = static_cast<__bf16>(p);
        }
        pb[2 * kt + sp] = v;
      }
    l_run = l_run * alpha + psum;
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[d][r] *= alpha;

    // ---- O^T += V^T P^T ----
#pragma unroll
    for (int S = 0; S < 4; ++S) {
      const int r0 = 16 * S + trow_base;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int ch = tch_base + 4 * db;
        const int offa = r0 * 256 + 16 * swz(r0, ch) + tbyte;
        const int offb = (r0 + 8) * 256 + 16 * swz(r0 + 8, ch) + tbyte;
        bf16x8 vf = tr_read_pair(vb, offa, offb);
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pb[S], o[db], 0, 0, 0);
      }
    }

    if (t + 1 < ntiles) stage_write(buf ^ 1);
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
  hipLaunchKernelGGL(attn_fwd_d128, dim3((unsigned)nwg), dim3(kThreads), 0, stream, a);
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}
