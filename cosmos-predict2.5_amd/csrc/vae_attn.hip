// Flash attention for the Wan VAE AttentionBlock (gfx950): one head of dimension 384, bf16 in / out.
//
//   cp25_vae_attn : O = softmax(Q K^T / sqrt(384)) V per frame, Q/K/V rows taken from strided buffers (the
//                   to_qkv output [T][L][3C] directly), replacing F.scaled_dot_product_attention in
//                   AttentionBlock.forward (cosmos_predict2/_src/predict2/tokenizers/wan2pt1.py:225-261,
//                   q, k, v = [b*t, 1, h*w, c], one head) and the S = QK^T / softmax / PV round trip the
//                   round-1 build made through HBM (a 14 080^2 fp32 score matrix per frame at 704 x 1280).
//
// Design: one workgroup = 4 waves (one per SIMD) = 128 query rows; every wave owns 32 rows and the
// whole head dimension:
//   * swapped products as in attn_fwd.hip: S^T = K Q^T (v_mfma_f32_32x32x16_bf16, 24 k-steps over d; the
//     query on the lane, Q^T fragments resident in 96 VGPRs), then O^T = V^T P^T with the S accumulator
//     converted to bf16 in place as the B operand and V^T read by ds_read_b64_tr_b16; O^T is 12 d-blocks of
//     32 x 32 (192 accumulators);
//   * two passes over the keys: the exact row max (Q K^T only), then P = exp2(S c - m) with that fixed shift,
//     so O^T is never rescaled and stays in the accumulator file (192 registers next to the 96 of Q^T);
//     P rounded to bf16 for P V as flash kernels do;
//   * K/V stream through LDS in 32-key tiles (24 KB each), double-buffered, register-staged by all 256
//     threads one tile ahead; padded rows (K 784 B, V 832 B) keep the K row reads and the transposed V reads
//     bank-conflict-free (the same padding rule as attn_fwd.hip's 272 / 320 B rows at d = 128).
//   * when the query blocks alone do not cover the CUs (one frame: 110 blocks), the keys are split over up to
//     8 workgroups per block (flash-decoding); each writes (O, m, l) partials and vae_attn_combine merges them.
// Numerics: fp32 scores / max / sum, bf16 P, fp32 O normalised once and rounded to bf16 (the same values a
// one-pass online softmax reaches once its running max is final).
#include "cp25_common.h"

namespace {

constexpr int kVD = 384;            // head dim
constexpr int kVKS = kVD / 16;      // 24 k-steps of 16 over d
constexpr int kVDB = kVD / 32;      // 12 d-blocks of 32
constexpr int kVKeys = 32;          // keys per tile
constexpr int kVKStride = kVD * 2 + 16;   // 784
constexpr int kVVStride = kVD * 2 + 64;   // 832
constexpr int kVKBuf = kVKeys * kVKStride;  // 25088
constexpr int kVVBuf = kVKeys * kVVStride;  // 26624
constexpr int kVStage = kVKBuf + kVVBuf;
constexpr int kVChunks = kVKeys * kVD / 8;  // 16-B chunks per K (or V) tile: 1536
constexpr int kVPerThread = kVChunks / 256;  // 6

struct VaeAttnArgs {
  const unsigned short* q;
  const unsigned short* k;
  const unsigned short* v;
  unsigned short* o;
  int64_t ldq, ldk, ldv, ldo;          // row strides (elements)
  int64_t fq, fk, fv, fo;              // frame strides (elements)
  int Lq, Lk;
  float scale_log2;                    // softmax scale * log2(e)
  int splits;                          // key splits (grid.z): > 1 writes partials to ws for vae_attn_combine
  float* ws;                           // [splits][T][Lq][D + 2] fp32: O (unnormalised), m, l
};

__global__ void __launch_bounds__(256, 1) vae_attn_kernel(VaeAttnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kVStage];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l31 = lane & 31, hl = lane >> 5;
  const int frame = blockIdx.y;
  const unsigned short* Q = a.q + frame * a.fq;
  const unsigned short* K = a.k + frame * a.fk;
  const unsigned short* V = a.v + frame * a.fv;
  unsigned short* O = a.o + frame * a.fo;
  const int q0 = blockIdx.x * 128 + wave * 32;
  // this workgroup's key tiles: split blockIdx.z of a.splits (flash-decoding: more workgroups than query blocks)
  const int nt_all = (a.Lk + kVKeys - 1) / kVKeys;
  const int t_begin = (int)((int64_t)nt_all * blockIdx.z / a.splits);
  const int t_end = (int)((int64_t)nt_all * (blockIdx.z + 1) / a.splits);

  // Q^T fragments (B operand of S^T = K Q^T): lane (query l31, d 16 s + 8 hl .. + 8), 96 VGPRs
  bf16x8 qf[kVKS];
  {
    const int qr = min(q0 + l31, a.Lq - 1);  // rows past Lq repeat the last query (not stored)
#pragma unroll
    for (int s = 0; s < kVKS; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(Q + (int64_t)qr * a.ldq + 16 * s + 8 * hl);
  }

  // staging: thread t moves chunks t + 256 i (i < 6) of the K (and V) tile: row c / 48, 16-B chunk c % 48.
  // Rows past Lk repeat the last key (no branch): their scores are masked to -inf, so P = 0 for them.
  u32x4 sk[kVPerThread], sv[kVPerThread];
  auto load_tile = [&](int t, bool with_v) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < kVPerThread; ++i) {
      const int c = tid + 256 * i;
      const int key = min(t * kVKeys + c / (kVD / 8), a.Lk - 1);
      const int ch = c % (kVD / 8);
      sk[i] = *reinterpret_cast<const u32x4*>(K + (int64_t)key * a.ldk + ch * 8);
      if (with_v) sv[i] = *reinterpret_cast<const u32x4*>(V + (int64_t)key * a.ldv + ch * 8);
    }
  };
  auto write_tile = [&](int buf, bool with_v) __attribute__((always_inline)) {
    char* kb = smem + buf * kVStage;
    char* vb = kb + kVKBuf;
#pragma unroll
    for (int i = 0; i < kVPerThread; ++i) {
      const int c = tid + 256 * i;
      const int r = c / (kVD / 8), ch = c % (kVD / 8);
      *reinterpret_cast<u32x4*>(kb + r * kVKStride + ch * 16) = sk[i];
      if (with_v) *reinterpret_cast<u32x4*>(vb + r * kVVStride + ch * 16) = sv[i];
    }
  };

  // per-lane LDS read offsets: K rows (key l31, d 16 s + 8 hl); V^T transposed reads as attn_fwd.hip
  const int k_rd = l31 * kVKStride + 16 * hl;
  const int grp = lane >> 4, gi = lane & 15;
  const int tq = gi >> 2, tp = gi & 3;
  const int v_rd = kVKBuf + (4 * (grp >> 1) + tq) * kVVStride + 32 * (grp & 1) + 8 * tp;

  // S^T of one tile, operand reads two MFMAs ahead into a 3-deep ring (the fences keep the compiler from hoisting
  // all 24 reads, 96 VGPRs, to the top); keys past Lk -> -inf (register r of the lane holds key 8 (r / 4) + 4 hl
  // + r % 4 of the tile)
  auto scores = [&](const char* kb, int t) __attribute__((always_inline)) {
    f32x16 S;
#pragma unroll
    for (int r = 0; r < 16; ++r) S[r] = 0.f;
    bf16x8 kr[3];
    kr[0] = *reinterpret_cast<const bf16x8*>(kb + k_rd);
    kr[1] = *reinterpret_cast<const bf16x8*>(kb + k_rd + 32);
#pragma unroll
    for (int s = 0; s < kVKS; ++s) {
      if (s + 2 < kVKS) kr[(s + 2) % 3] = *reinterpret_cast<const bf16x8*>(kb + k_rd + 32 * (s + 2));
      S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kr[s % 3], qf[s], S, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if ((t + 1) * kVKeys > a.Lk) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (t * kVKeys + 8 * (r >> 2) + 4 * hl + (r & 3) >= a.Lk) S[r] = -INFINITY;
    }
    return S;
  };

  // ---- pass 1: the exact row max over all keys (Q K^T only). With it fixed, pass 2 never rescales O, so O stays
  // in the accumulator file and is touched only by MFMAs (a running-max rescale would need all 192 values in
  // VGPRs next to the Q^T fragments). Costs 1.5x the MFMAs of a single pass; the round-1 path's 793 MB score
  // matrix per frame is gone.
  float mx = -INFINITY;
  load_tile(t_begin, false);
  write_tile(0, false);
  __syncthreads();
  for (int t = t_begin; t < t_end; ++t) {
    const int buf = (t - t_begin) & 1;
    if (t + 1 < t_end) load_tile(t + 1, false);
    const f32x16 S = scores(smem + buf * kVStage, t);
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, S[r]);
    if (t + 1 < t_end) write_tile(buf ^ 1, false);  // tile t - 1's buffer: every wave passed the last barrier
    __syncthreads();
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  const float m_row = mx * a.scale_log2;

  // ---- pass 2: P = exp2(S c - m), l += sum P, O^T += V^T P^T
  f32x16 o[kVDB];
#pragma unroll
  for (int d = 0; d < kVDB; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float l_run = 0.f;
  load_tile(t_begin, true);
  write_tile(0, true);
  __syncthreads();
  for (int t = t_begin; t < t_end; ++t) {
    const int buf = (t - t_begin) & 1;
    if (t + 1 < t_end) load_tile(t + 1, true);
    const f32x16 S = scores(smem + buf * kVStage, t);
    bf16x8 pb[2];
#pragma unroll
    for (int sp = 0; sp < 2; ++sp)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float p = __builtin_amdgcn_exp2f(fmaf(S[8 * sp + j], a.scale_log2, -m_row));
        l_run += p;
        pb[sp][j] = static_cast<__bf16>(p);
      }
    const char* vb = smem + buf * kVStage + v_rd;
    auto v_frag = [&](int ks, int d) __attribute__((always_inline)) {
      typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
      typedef __attribute__((address_space(3))) const char* lds_cptr;
      const int off = 16 * ks * kVVStride + 64 * d;
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds_cptr)(vb + off));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds_cptr)(vb + off + 8 * kVVStride));
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      const s16x8 r8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, r8);
    };
    bf16x8 vr[3];
    vr[0] = v_frag(0, 0);
    vr[1] = v_frag(0, 1);
#pragma unroll
    for (int i = 0; i < 2 * kVDB; ++i) {
      if (i + 2 < 2 * kVDB) vr[(i + 2) % 3] = v_frag((i + 2) / kVDB, (i + 2) % kVDB);
      o[i % kVDB] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vr[i % 3], pb[i / kVDB], o[i % kVDB], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (t + 1 < t_end) write_tile(buf ^ 1, true);
    __syncthreads();
  }

  // ---- epilogue: O^T lane (query l31), register r of d-block d holds d = 32 d + 8 (r / 4) + 4 hl + r % 4
  const float l_tot = l_run + __shfl_xor(l_run, 32);
  const int qr = q0 + l31;
  if (qr >= a.Lq) return;
  if (a.splits > 1) {  // partial (O unnormalised, m, l) for vae_attn_combine
    float* wrow = a.ws + (((int64_t)blockIdx.z * gridDim.y + frame) * a.Lq + qr) * (kVD + 2);
#pragma unroll
    for (int d = 0; d < kVDB; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 w = {o[d][4 * g], o[d][4 * g + 1], o[d][4 * g + 2], o[d][4 * g + 3]};
        *reinterpret_cast<f32x4*>(wrow + 32 * d + 8 * g + 4 * hl) = w;
      }
    if (hl == 0) {
      wrow[kVD] = m_row;
      wrow[kVD + 1] = l_tot;
    }
    return;
  }
  const float inv = 1.f / l_tot;
  unsigned short* orow = O + (int64_t)qr * a.ldo;
#pragma unroll
  for (int d = 0; d < kVDB; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      u16x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = f2bf(o[d][4 * g + e] * inv);
      *reinterpret_cast<u16x4*>(orow + 32 * d + 8 * g + 4 * hl) = w;
    }
}

// out[t][q] = sum_s w_s O_s / sum_s w_s l_s, w_s = exp2(m_s - max_s m_s): one wave per query row
__global__ void __launch_bounds__(256) vae_attn_combine(const float* __restrict__ ws, int splits, int T, int Lq,
                                                        unsigned short* __restrict__ o, int64_t ldo, int64_t fo) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T * Lq) return;
  const int t = row / Lq, q = row % Lq;
  const int64_t rs = (int64_t)T * Lq * (kVD + 2);  // split stride
  const float* w0 = ws + (int64_t)row * (kVD + 2);
  float m = -INFINITY;
  for (int s = 0; s < splits; ++s) m = fmaxf(m, w0[s * rs + kVD]);
  float acc[kVD / 64] = {};
  float l = 0.f;
  for (int s = 0; s < splits; ++s) {
    const float* w = w0 + s * rs;
    const float f = __builtin_amdgcn_exp2f(w[kVD] - m);
    l += f * w[kVD + 1];
#pragma unroll
    for (int i = 0; i < kVD / 64; ++i) acc[i] += f * w[i * 64 + lane];
  }
  const float inv = 1.f / l;
  unsigned short* orow = o + t * fo + (int64_t)q * ldo;
#pragma unroll
  for (int i = 0; i < kVD / 64; ++i) orow[i * 64 + lane] = f2bf(acc[i] * inv);
}

// key splits: enough workgroups to cover the CUs when the query blocks alone do not (one frame at 704 x 1280
// has 110 blocks of 128 queries for 256 CUs), at least 8 key tiles per split
int vae_attn_splits(int T, int Lq, int Lk) {
  const int blocks = (int)cdiv(Lq, 128) * T;
  const int tiles = (int)cdiv(Lk, kVKeys);
  int s = 1;
  while (s < 8 && blocks * (s + 1) <= 320 && tiles / (s + 1) >= 8) ++s;
  return s;
}

}  // namespace

extern "C" int64_t cp25_vae_attn_workspace_bytes(int T, int Lq, int Lk, int D) {
  if (T <= 0 || Lq <= 0 || Lk <= 0 || D != kVD) return 0;
  const int s = vae_attn_splits(T, Lq, Lk);
  return s > 1 ? (int64_t)s * T * Lq * (kVD + 2) * 4 : 0;
}

extern "C" int cp25_vae_attn(const void* q, int64_t ldq, int64_t fq, const void* k, int64_t ldk, int64_t fk,
                             const void* v, int64_t ldv, int64_t fv, void* o, int64_t ldo, int64_t fo, int T, int Lq,
                             int Lk, int D, float scale, void* workspace, int64_t workspace_bytes,
                             hipStream_t stream) {
  if (!q || !k || !v || !o || T <= 0 || Lq <= 0 || Lk <= 0 || !(scale > 0.f)) return CP25_ERR_INVAL;
  if (D != kVD) return CP25_ERR_DTYPE;
  if (ldq < D || ldk < D || ldv < D || ldo < D || (ldq | ldk | ldv | ldo | fq | fk | fv | fo) % 8) return CP25_ERR_INVAL;
  if ((((uintptr_t)q) | ((uintptr_t)k) | ((uintptr_t)v) | ((uintptr_t)o)) & 15) return CP25_ERR_INVAL;
  if (T > 65535) return CP25_ERR_INVAL;
  const int splits = vae_attn_splits(T, Lq, Lk);
  if (splits > 1 && (!workspace || workspace_bytes < cp25_vae_attn_workspace_bytes(T, Lq, Lk, D) ||
                     ((uintptr_t)workspace & 15)))
    return CP25_ERR_INVAL;
  VaeAttnArgs a;
  a.q = (const unsigned short*)q;
  a.k = (const unsigned short*)k;
  a.v = (const unsigned short*)v;
  a.o = (unsigned short*)o;
  a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo;
  a.fq = fq; a.fk = fk; a.fv = fv; a.fo = fo;
  a.Lq = Lq; a.Lk = Lk;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.splits = splits;
  a.ws = (float*)workspace;
  hipLaunchKernelGGL(vae_attn_kernel, dim3((unsigned)cdiv(Lq, 128), (unsigned)T, (unsigned)splits), dim3(256), 0,
                     stream, a);
  CP25_LAUNCH_CHECK();
  if (splits > 1) {
    hipLaunchKernelGGL(vae_attn_combine, dim3((unsigned)cdiv((int64_t)T * Lq, 4)), dim3(256), 0, stream,
                       (const float*)workspace, splits, T, Lq, (unsigned short*)o, ldo, fo);
    CP25_LAUNCH_CHECK();
  }
  return CP25_OK;
}
