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
//   * one pass over the keys with the softmax shift fixed at the first key tile's row max, so O^T is never
//     rescaled and stays in the accumulator file (192 registers next to the 96 of Q^T); a workgroup whose rows see
//     a later tile max more than 2^24 above that shift redoes its block with the exact row max of all keys (a
//     Q K^T-only pass first, round 3's form); P rounded to bf16 for P V as flash kernels do;
//   * K/V stream through LDS in 32-key tiles (24 KB each), double-buffered, register-staged by all 256
//     threads one tile ahead; padded rows (K 784 B, V 832 B) keep the K row reads and the transposed V reads
//     bank-conflict-free (the same padding rule as attn_fwd.hip's 272 / 320 B rows at d = 128).
//   * when the query blocks alone do not cover the CUs (one frame: 110 blocks), the keys are split over up to
//     8 workgroups per block (flash-decoding); each writes (O, m, l) partials and vae_attn_combine merges them.
// Numerics: fp32 scores / max / sum, bf16 P (terms <= 2^24 after the shift), fp32 O normalised once and rounded to
// bf16.
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
constexpr float kVLazy = 24.f;              // one-pass form: largest exponent a term may reach past the first tile's max

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
  int* flags;                          // [splits][T][query blocks]: the one-pass form overflowed (kFix redoes)
};

// kFix = false: the one-pass form; a workgroup whose first-tile shift a later tile overflows writes flags[wg] = 1 and
// no output. kFix = true (launched next on the same stream): such workgroups (any other exits at once) redo the block
// with the exact row max of all keys (a Q K^T-only pass, then the P V pass with that shift).
template <bool kFix>
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
  const int64_t wg = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  if constexpr (kFix) {
    if (a.flags[wg] == 0) return;  // the one-pass launch finished this block
  }

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

  // ---- P V pass: P = exp2(S c - m), l += sum P, O^T += V^T P^T with a shift m fixed for the whole pass, so O is
  // never rescaled and stays in the accumulator file (a rescale of the 192 accumulators inside the loop spilled).
  // kOnline: m is the first tile's row max, and the pass reports (wave-uniform) whether a later tile's row max
  // exceeded it by more than kVLazy (P would pass 2^24): then the kFix launch redoes the block with the exact row max
  // of all keys (a Q K^T-only pass first, 1.5x the MFMAs, round 3's only form). Keys of one frame rarely do. (The
  // redo inside the same kernel spilled: two inlined copies of this pass.)
  f32x16 o[kVDB];
  float l_run = 0.f, m_row = -INFINITY;
  auto pv_pass = [&](auto online_c) __attribute__((always_inline)) {
    constexpr bool kOnline = decltype(online_c)::value;
    bool ovf = false;
#pragma unroll
    for (int d = 0; d < kVDB; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
    l_run = 0.f;
    load_tile(t_begin, true);
    write_tile(0, true);
    __syncthreads();
    for (int t = t_begin; t < t_end; ++t) {
      const int buf = (t - t_begin) & 1;
      if (t + 1 < t_end) load_tile(t + 1, true);
      const f32x16 S = scores(smem + buf * kVStage, t);
      if constexpr (kOnline) {
        float tmax = S[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) tmax = fmaxf(tmax, S[r]);
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32)) * a.scale_log2;  // the row's (lanes l31, l31 + 32) tile max
        if (t == t_begin)
          m_row = tmax;
        else
          ovf = ovf || __any(tmax > m_row + kVLazy);
      }
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
    return ovf;
  };

  if constexpr (!kFix) {
    __shared__ int redo;     // any wave of the workgroup overflowed the first-tile shift
    if (tid == 0) redo = 0;  // ordered before the waves' writes by the pass's first barrier
    const bool ovf = pv_pass(std::true_type{});
    if (ovf && lane == 0) redo = 1;
    __syncthreads();
    if (tid == 0) a.flags[wg] = redo;
    if (redo) return;  // the kFix launch writes this block
  } else {
    // the exact row max over all keys (Q K^T only), then the P V pass with it
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
    m_row = mx * a.scale_log2;
    pv_pass(std::false_type{});
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

// workspace: the per-workgroup overflow flags (rounded to 256 B), then the key-split partials when splits > 1
static int64_t vae_attn_flag_bytes(int T, int Lq, int Lk) {
  return ((int64_t)vae_attn_splits(T, Lq, Lk) * T * cdiv(Lq, 128) * 4 + 255) / 256 * 256;
}

extern "C" int64_t cp25_vae_attn_workspace_bytes(int T, int Lq, int Lk, int D) {
  if (T <= 0 || Lq <= 0 || Lk <= 0 || D != kVD) return 0;
  const int s = vae_attn_splits(T, Lq, Lk);
  return vae_attn_flag_bytes(T, Lq, Lk) + (s > 1 ? (int64_t)s * T * Lq * (kVD + 2) * 4 : 0);
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
  if (!workspace || workspace_bytes < cp25_vae_attn_workspace_bytes(T, Lq, Lk, D) || ((uintptr_t)workspace & 15))
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
  a.flags = (int*)workspace;
  a.ws = (float*)((char*)workspace + vae_attn_flag_bytes(T, Lq, Lk));
  const dim3 grid((unsigned)cdiv(Lq, 128), (unsigned)T, (unsigned)splits);
  hipLaunchKernelGGL(vae_attn_kernel<false>, grid, dim3(256), 0, stream, a);
  CP25_LAUNCH_CHECK();
  hipLaunchKernelGGL(vae_attn_kernel<true>, grid, dim3(256), 0, stream, a);
  CP25_LAUNCH_CHECK();
  if (splits > 1) {
    hipLaunchKernelGGL(vae_attn_combine, dim3((unsigned)cdiv((int64_t)T * Lq, 4)), dim3(256), 0, stream,
                       (const float*)a.ws, splits, T, Lq, (unsigned short*)o, ldo, fo);
    CP25_LAUNCH_CHECK();
  }
  return CP25_OK;
}
