// Flash-attention forward for the DiT self- and cross-attention (gfx950, bf16 in/out, head dim 128).
//
// Replaces the reference's attention op: cosmos_predict2/_src/predict2/networks/attention.py:90-181
// (q/k/v recast to bf16, softmax(QK^T / sqrt(D)) V, no mask, no dropout, non-causal), which the DiT
// calls through MinimalA2AAttnOp (networks/a2a_cp.py:208-219) on [B, S, H, D] tensors.
//
// Design (MI355X-first, see DESIGN.md "attn_fwd"):
//   * one workgroup = 8 waves = 256 query rows of one (batch, head); every wave owns 32 query rows;
//   * "swapped" products so the softmax is lane-local: S^T = K Q^T (v_mfma_f32_32x32x16_bf16, the
//     query on the lane), then O^T = V^T P^T, whose B operand is the S accumulator converted to bf16
//     with no lane movement, and whose A operand (V^T) comes from ds_read_b64_tr_b16 (hardware
//     transposed LDS read) of the row-major V tile;
//   * ping-pong between the two waves of each SIMD (comment above attn_fwd_d128): one runs its 32
//     MFMAs of a tile while the other runs its softmax, swapping at every barrier;
//   * the MFMA phase's LDS operand reads are issued four MFMAs ahead (inline asm, counted lgkmcnt);
//   * K/V stream through LDS in 64-key tiles, double buffered, register-staged by buffer_load with
//     a wave-uniform descriptor (the hardware range check zero-fills rows past the end);
//   * padded LDS rows (K 272 B, V 320 B) keep both the ds_read_b128 row reads of K and the transposed
//     reads of V bank-conflict-free with every address a per-lane base + immediate;
//   * the O rescale of the online softmax is skipped (exactly) when no row max of the wave grew;
//   * bounded shift (cp25_attn_fwd_bounded): given bounds on the query and key norms, every score of
//     query row q lies in [-b, b] with b = |q_row| max|k| * scale (Cauchy-Schwarz, log2 units), so a
//     fixed per-row shift m = max(b - kTop, 0) replaces the running max: the softmax has no max
//     reduction, no rescale and no max -> exp dependency. Softmax is shift invariant, so this is the
//     same result up to rounding, as long as every term stays in range: s - m <= kTop (no overflow of
//     the row sum) and the row's largest term >= 2^(-b - m) >= 2^-100 (the row max is >= -b). Both
//     hold for b <= kMaxBound; the host launches this form only when max|q| max|k| * scale is under it;
//   * grid remapped so the workgroups of one XCD share a (batch, head): their K/V stream hits in
//     that XCD's L2 instead of HBM.
// NaN inputs are not supported (built with -fno-honor-nans; the reference's flash kernels do not
// define NaN propagation either).
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
constexpr float kTop = 60.f;        // bounded shift: largest exponent a term may reach (log2 units)
constexpr float kMaxBound = 80.f;   // bounded shift: largest score bound b (2 b - kTop <= 100)
// LDS layout (bytes): [K0 | K1 | V0 | V1]. Padded rows instead of an XOR swizzle so every LDS read
// is one per-lane base VGPR + a compile-time immediate (no per-tile address arithmetic):
//   K rows 272 B (256 + 16): the 16 rows a ds_read_b128 lane group reads at one column land on 16
//     distinct 16-B bank slots;
//   V rows 320 B (256 + 64): the 4 rows x 64 B a half-wave of ds_read_b64_tr_b16 reads land on the
//     4 distinct 64-B quarters of the 256-B bank row.
constexpr int kKStride = 272;
constexpr int kVStride = 320;
constexpr int kVBuf = kKBlk * kVStride;  // 20480
constexpr int kKBuf = kKBlk * kKStride;  // 17408
constexpr int kLdsBytes = 2 * kVBuf + 2 * kKBuf;  // 75776

typedef __attribute__((address_space(3))) s16x4* lds_s16x4_ptr;
typedef __attribute__((address_space(3))) const char* lds_char_ptr;

// compile-time loop: f(integral_constant<int, I>) for I = 0 .. N-1, in order
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
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
  int nsplit;       // key-range splits per (b, h, query block) (1: O written directly)
  int tps;          // key tiles per split
  int nchunk;       // persistent short-KV form: workgroups per (b, h), each a contiguous run of query blocks
  int ntk_v;        // fp8 P.V: key tiles per (b, h) of the v8t layout (ceil(Lk / 64))
  const float* v_amax;  // fp8 P.V: per-(b, h) max |v| (v8t holds v * 448 / amax)
  float s_init;     // fp8 P.V: the Q K^T chains' initial C (-shift: P = exp2(S - shift) <= 2^15 fits e5m2)
  float* o_part;    // nsplit > 1: [nsplit][B][H][Lq][128] fp32 partial O (normalised per split)
  float* lse_part;  // nsplit > 1: [nsplit][B][H][Lq] fp32 log2-sum-exp2 of the scaled scores
  float scale_log2; // softmax scale * log2(e)
  float kbound;     // > 0: upper bound of |k| over all keys (bounded shift); 0: online max only
#ifdef CP25_ATTN_PROBE
  unsigned long long* probe;  // [wg < 8][wave][tile - probe_t0 < 32][8] s_memtime stamps (lab build only)
  int probe_t0;
#endif
};

// Lab-build instrumentation (tools/attn_probe.py): s_memtime around the two barriers of a tile
// iteration for the first 8 workgroups; compiled out of the product library.
#ifdef CP25_ATTN_PROBE
#define ATTN_STAMP(t, k)                                                                              \
  do {                                                                                                \
    const int pt_ = (t) - a.probe_t0;                                                                 \
    if (a.probe && blockIdx.x < 8 && pt_ >= 0 && pt_ < 32)                                                 \
      a.probe[(((size_t)blockIdx.x * kWaves + wave) * 32 + pt_) * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define ATTN_STAMP(t, k) do { } while (0)
#endif

// Ping-pong schedule. Waves w and w+4 share a SIMD; the workgroup's waves split into group A
// (waves 0-3) and group B (waves 4-7) that run opposite phases between the same barriers:
//
//   phase 2t  : A  MFMA  S = K(t+1) Q^T,  O^T += V(t)^T P(t)^T        B  softmax S(t) -> P(t), stage K
//   phase 2t+1: A  softmax S(t+1) -> P(t+1), stage V                  B  MFMA (same products as A's)
//
// so every SIMD has one wave feeding the matrix pipe (32 back-to-back MFMAs) while its partner runs
// the exp/max/sum VALU work in the issue slots the MFMAs leave free. K/V tiles are double buffered in
// LDS; group B stages K (register-staged, loads issued two phases before their LDS write), group A
// stages V. Buffer lifetimes: K(j) and V(j) live in buffer j&1; K(t+1), V(t) are read in phases 2t
// and 2t+1; K(t+2) is written in phase 2t over K(t) (last read in 2t-1), V(t+1) in phase 2t+1 over
// V(t-1) (last read in 2t-1).
// kKind 0: self-attention, 1: cross-attention (separate symbols in profiles); kFixed: bounded shift;
// kPre: q pre-scaled by scale * log2(e) and |q| |k| <= kTop (host-checked): P = exp2(S), shift 0
// kF8 >= 1 (cp25_attn_fwd_prescaled_fp8qk, the config-5 fp8 option): q and k arrive as OCP e4m3 (bytes, strides
// in bytes) and S^T = K Q^T runs on v_mfma_f32_32x32x64_f8f6f4: 4 MFMAs of 64 k per tile instead of 16 of 16,
// K tiles of 64 rows x 128 B (LDS rows 144 B). The operand k order only has to agree between A and B: lane half
// h, byte i of both operands is d = 64 s + 32 h + i. kF8 = 2 (cp25_attn_fwd_prescaled_fp8) also runs O^T += V^T
// P^T there: P as e5m2 straight from the S^T accumulator (byte j = 16 kt + r), V^T as e4m3 from the v8t layout
// (cp25_cast_v_fp8t: per-(b, h) scale, keys permuted to the P bytes), 4 MFMAs per tile instead of 16, LDS V rows
// of 64 B padded to 80. The shift that keeps P = exp2(S - shift) <= 2^15 enters as the Q K^T chains' initial C.
// kF8 = 3 makes the e5m2 byte of P without exp2: n = round(4 (S - shift) + 60) clamped to [0, 255] by one
// v_cvt_pk_u8_f32 (after one fma) is read as e5m2, i.e. 2^(n / 4 - 15) with a linear mantissa, and the row sums
// come from a fifth P.V MFMA against an all-ones V^T row (so they are the sums of the P actually used).
// kPersist (cross-attention, Lk <= 1024, cp25_attn_fwd_prescaled): one workgroup per CU runs a contiguous run of
// query blocks of one (b, h) as one stream of key tiles (tile t = key tile t % ntk of block t / ntk). The
// pipeline never drains between blocks: after the MFMA phase that closes a block, the wave stores that block's
// O (and zeroes it) in its next VALU phase, and Q of the next block is reloaded right after the phase that ran
// the old Q's last Q K^T. Without it, the 8 key tiles of a 512-key cross-attention paid the whole per-workgroup
// prologue / epilogue (about 44 tiles of fixed cost, plan_split's fitted model) for every 256 queries.
template <int kKind, bool kFixed, bool kPre = false, int kF8 = 0, bool kPersist = false>
__global__ void __launch_bounds__(kThreads, 2) attn_fwd_d128(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];
  static_assert(!kF8 || kPre, "the fp8 Q K^T form is the prescaled one");
  static_assert(!kPersist || (kPre && !kF8), "the persistent form is the prescaled bf16 one");
  static_assert(kF8 >= 0 && kF8 <= 3, "kF8: 0 bf16, 1 fp8 Q K^T, 2 + fp8 P.V, 3 + P bytes without exp2");
  constexpr int KSTR = kF8 ? 144 : kKStride;        // K LDS row stride
  constexpr int KB1 = kKBlk * KSTR;                 // K buffer 1
  constexpr int VB0 = 2 * kKBlk * KSTR, VB1 = VB0 + kVBuf;
  typedef int i32x8 __attribute__((ext_vector_type(8)));

  const int nwg = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, nwg);
  // tile order (b, h) > split > query block: an XCD's contiguous tile range streams one key range
  const int qb = kPersist ? (int)((int64_t)(tile % a.nchunk) * a.nqb / a.nchunk) : tile % a.nqb;
  const int bhs = kPersist ? tile / a.nchunk : tile / a.nqb;
  const int split = kPersist ? 0 : bhs % a.nsplit, bh = kPersist ? bhs : bhs / a.nsplit;
  const int nblk = kPersist ? (int)((int64_t)(tile % a.nchunk + 1) * a.nqb / a.nchunk) - qb : 1;
  const int b = bh / a.H, h = bh % a.H;
  // this workgroup's keys: [split * tps * 64, ...) as a self-contained key sequence of length Lk
  const int key0 = split * a.tps * kKBlk;
  const int Lk = min(a.Lk - key0, a.tps * kKBlk);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int l31 = lane & 31;
  const int hl = lane >> 5;  // lane half
  const bool group_b = __builtin_amdgcn_readfirstlane(tid) >= kThreads / 2;

  constexpr int QKE = kF8 ? 1 : 2;  // bytes per q / k element
  const char* qp = (const char*)a.q + (b * a.q_sb + h * a.q_sh) * QKE;
  const char* kp = (const char*)a.k + (b * a.k_sb + h * a.k_sh + (int64_t)key0 * a.k_sl) * QKE;
  const unsigned short* vp = kF8 >= 2 ? (const unsigned short*)((const char*)a.v + ((int64_t)bh * a.ntk_v + key0 / kKBlk) * 8192)
                                      : a.v + b * a.v_sb + h * a.v_sh + (int64_t)key0 * a.v_sl;

  // ---- Q fragments (B operand of S^T = K Q^T): Q[q][16s + 8hl .. +7], s = 0..7 ----
  const int q_row = qb * kQBlk + wave * kQRows + l31;
  const int q_row_c = q_row < a.Lq ? q_row : a.Lq - 1;
  bf16x8 qf[8];
  i32x8 qf8[2];
  if constexpr (kF8) {
    const char* src = qp + (int64_t)q_row_c * a.q_sl + 32 * hl;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const u32x4 lo = *reinterpret_cast<const u32x4*>(src + 64 * s);
      const u32x4 hi = *reinterpret_cast<const u32x4*>(src + 64 * s + 16);
      qf8[s] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
  } else {
    const char* src = qp + ((int64_t)q_row_c * a.q_sl + 8 * hl) * 2;
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(src + 32 * s);
  }

  f32x16 o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m_run = -1e30f;
  float l_run = 0.f;
  // bounded shift: m = |q_row| * kbound * scale_log2 (the host checked the cap on the norm bounds)
  if constexpr (kPre) {
    m_run = 0.f;
  } else if constexpr (kFixed) {
    float qq = 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = static_cast<float>(qf[s][e]);
        qq = fmaf(x, x, qq);
      }
    qq = wave_swap_sum(qq);  // the row's two lanes hold its two halves
    m_run = fmaxf(sqrtf(qq) * a.kbound * a.scale_log2 - kTop, 0.f);
  }

  const int ntk = (Lk + kKBlk - 1) / kKBlk;       // key tiles per query block
  const int ntiles = kPersist ? nblk * ntk : ntk;  // key tiles this workgroup streams

  // staging: a group's 256 threads own 4 chunks (16 B) each of a 64x128 tile: rows u/16 + 16 i,
  // chunk u%16. buffer_load: the tile base is a wave-uniform descriptor (SALU only), the per-lane
  // offset is loop-invariant, rows past Lk fall outside the descriptor's range and read as zero
  // (their scores are masked to -inf).
  // kF8: a K tile is 64 rows x 128 B, 2 chunks of 16 B per thread of group B (rows u/8 + 32 i, chunk u%8)
  // kF8 == 2: a V tile is 128 d rows x 64 B (8 KiB contiguous in v8t), 2 chunks per thread of group A (rows u/4 +
  // 64 i, chunk u%4); always whole (v8t pads the last tile with zero keys)
  const int u = tid & (kThreads / 2 - 1);
  const bool kf8 = kF8 && group_b;
  const bool v8 = kF8 >= 2 && !group_b;
  const int srow = kf8 ? u >> 3 : (v8 ? u >> 2 : u >> 4), sch = kf8 ? u & 7 : (v8 ? u & 3 : u & 15);
  const int64_t sl = group_b ? a.k_sl : (v8 ? 64 : a.v_sl);
  const int esz = (kf8 || v8) ? 1 : 2;
  const char* sbase = group_b ? kp : (const char*)vp;
  const int st_off = (int)(srow * sl * esz) + sch * 16, st_step = (int)((kf8 ? 32 : (v8 ? 64 : 16)) * sl * esz);
  const int nst = (kf8 || v8) ? 2 : 4;
  u32x4 st[4];
  auto load_tile = [&](int tt) __attribute__((always_inline)) {
    const int t = kPersist ? tt % ntk : tt;
    const int rows = min(Lk - t * kKBlk, kKBlk);
    const int nbytes = v8 ? (rows > 0 ? 8192 : 0) : (rows > 0 ? (int)((rows - 1) * sl * esz) + esz * kD : 0);
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(sbase + (int64_t)t * (v8 ? 8192 : kKBlk * sl * esz)), (short)0, nbytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < nst)
        st[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, st_off + i * st_step, 0, 0));
  };
  char* const k_wr = smem + srow * KSTR + sch * 16;
  constexpr int VSTR8 = 80;  // kF8 == 2: LDS V^T row stride (64 B + 16: conflict-free ds_read_b128 of d rows)
  char* const v_wr = smem + srow * (kF8 >= 2 ? VSTR8 : kVStride) + sch * 16;
  auto write_k = [&](auto BUF) __attribute__((always_inline)) {
    constexpr int kb = decltype(BUF)::value ? KB1 : 0;
    if constexpr (kF8) {
#pragma unroll
      for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4*>(k_wr + kb + 32 * i * KSTR) = st[i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) *reinterpret_cast<u32x4*>(k_wr + kb + 16 * i * KSTR) = st[i];
    }
  };
  auto write_v = [&](auto BUF) __attribute__((always_inline)) {
    constexpr int vb = decltype(BUF)::value ? VB1 : VB0;
    if constexpr (kF8 >= 2) {
#pragma unroll
      for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4*>(v_wr + vb + 64 * i * VSTR8) = st[i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) *reinterpret_cast<u32x4*>(v_wr + vb + 16 * i * kVStride) = st[i];
    }
  };

  // per-lane LDS read bases (everything else is an immediate offset)
  const char* const k_rd = smem + l31 * KSTR + (kF8 ? 32 : 16) * hl;  // + kt*32 rows + (64 | 32) s bytes
  const int grp = lane >> 4, gi = lane & 15;
  const int tq = gi >> 2, tp = gi & 3;
  const char* const v_rd = smem + VB0 + (4 * (grp >> 1) + tq) * kVStride + 32 * (grp & 1) + 8 * tp;  // + rows, + 64 db
  // the same bases as 32-bit LDS addresses for the MFMA phase's asm reads (all offsets < 64 KiB)
  const unsigned k_rd_lds = (unsigned)(uintptr_t)(lds_char_ptr)k_rd;
  const unsigned v_rd_lds = (unsigned)(uintptr_t)(lds_char_ptr)v_rd;

  // ragged last tile: keys >= Lk get a -inf score (a uniform branch taken on that tile only)
  const int ragged_tile = (Lk % kKBlk) != 0 ? Lk / kKBlk : -1;

  f32x16 S[2];   // S^T of the tile awaiting its softmax
  bf16x8 pb[4];  // P^T of the tile awaiting its P.V
  i32x8 pb8;     // kF8 >= 2: the same as e5m2 bytes (byte j = P from S[j >> 4][j & 15])
  const f32x16 zero16 = {};
  f32x16 sinit;  // kF8 >= 2: -shift in every element (initial C of the Q K^T chains)
#pragma unroll
  for (int r = 0; r < 16; ++r) sinit[r] = kF8 >= 2 ? a.s_init : 0.f;
  f32x16 lsum = {};  // kF8 == 3: the row sums, from P^T against an all-ones V^T row (every row of the block equal)
  const i32x8 ones8 = {0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838,
                       0x38383838};  // e4m3 1.0
  // kF8 == 2: one V^T A fragment = 32 B of the d row 32 db + l31, bytes 32 hl .. (two ds_read_b128)
  const char* const v_rd8 = smem + VB0 + l31 * VSTR8 + 32 * hl;
  auto v_frag8 = [&](int vb, int db) __attribute__((always_inline)) {
    const u32x4 lo = *reinterpret_cast<const u32x4*>(v_rd8 + vb + 32 * db * VSTR8);
    const u32x4 hi = *reinterpret_cast<const u32x4*>(v_rd8 + vb + 32 * db * VSTR8 + 16);
    return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  };

  // S^T = K Q^T on the K buffer; the first MFMA of each chain takes an inline-constant zero C
  // fp8 form: one A fragment = 32 B of a K row (d 64 s + 32 hl ..), two ds_read_b128
  auto k_frag8 = [&](int kb, int kt, int s) __attribute__((always_inline)) {
    const u32x4 lo = *reinterpret_cast<const u32x4*>(k_rd + kb + kt * 32 * KSTR + 64 * s);
    const u32x4 hi = *reinterpret_cast<const u32x4*>(k_rd + kb + kt * 32 * KSTR + 64 * s + 16);
    return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  };
  auto qk_mma = [&](auto BUF) __attribute__((always_inline)) {
    constexpr int kb = decltype(BUF)::value ? KB1 : 0;
    if constexpr (kF8) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
          S[kt] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(k_frag8(kb, kt, s), qf8[s],
                                                                 s == 0 ? (kF8 >= 2 ? sinit : zero16) : S[kt],
                                                                 0, 0, 0, 0, 0, 0);
      return;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(k_rd + kb + kt * 32 * KSTR + 32 * s);
        S[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], s == 0 ? zero16 : S[kt], 0, 0, 0);
      }
  };
  // online softmax of tile t: running max (O rescale skipped exactly when no row max of the wave
  // grew), P = exp2(S c - m) -> bf16 (lane-local B operand of P.V), row sum
  auto softmax = [&](int tt) __attribute__((always_inline)) {
    const int t = kPersist ? tt % ntk : tt;
    if (__builtin_expect(t == ragged_tile, 0)) {
      // the keys left in this tile, opaque to the compiler: otherwise (t == ragged_tile is loop invariant) it
      // hoists all 32 lane masks out of the tile loop, 64 SGPRs that the persistent form spills
      if constexpr (kPersist) {
        int left = Lk - t * kKBlk - 4 * hl;
        asm volatile("" : "+v"(left));
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kt * 32 + (r & 3) + 8 * (r >> 2) >= left) S[kt][r] = -INFINITY;
      } else {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = t * kKBlk + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
            if (key >= Lk) S[kt][r] = -INFINITY;
          }
      }
    }
    // S enters here: keeps the (otherwise dependency-free) bounded-shift exp work from being
    // hoisted across the barrier into the MFMA phase, where it would double the live P registers
    asm volatile("" : "+v"(S[0]), "+v"(S[1]));
    if constexpr (!kFixed) {
      // four independent v_max3 chains (this file builds with -fno-honor-nans: no canonicalising
      // v_max before each fmaxf of an MFMA result)
      float mc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) mc[j] = fmaxf(S[0][j], S[1][j]);
#pragma unroll
      for (int r = 4; r < 16; ++r) mc[r & 3] = fmaxf(fmaxf(mc[r & 3], S[0][r]), S[1][r]);
      const float mx = wave_swap_max(fmaxf(fmaxf(fmaxf(mc[0], mc[1]), mc[2]), mc[3]));
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
    } else {
      // contract guard: a norm bound below the real norms can only show as an overflowed row sum
      // (moderate violations are still exact by shift invariance); poison the row (NaN) instead of
      // returning a silently wrong one. Never taken under the contract.
      if (__builtin_expect(__any(l_run > 3.0e38f), 0)) {
        const float nan = __uint_as_float(0x7fc00000u);
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[d][r] = nan;
      }
    }
    float psum = 0.f;
    if constexpr (kF8 == 3) {
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        unsigned x = 0u;
#pragma unroll
        for (int e = 0; e < 4; ++e) x = __builtin_amdgcn_cvt_pk_u8_f32(fmaf(S[w >> 2][4 * (w & 3) + e], 4.f, 60.f), e, x);
        pb8[w] = (int)x;
      }
      asm volatile("" ::"v"(pb8));
      return;
    }
    if constexpr (kF8 == 2) {
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        float p[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          p[e] = __builtin_amdgcn_exp2f(S[w >> 2][4 * (w & 3) + e]);
          psum += p[e];
        }
        int q = __builtin_amdgcn_cvt_pk_bf8_f32(p[0], p[1], 0, false);
        pb8[w] = __builtin_amdgcn_cvt_pk_bf8_f32(p[2], p[3], q, true);
      }
      l_run += psum;
      asm volatile("" ::"v"(pb8), "v"(l_run));
      return;
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float p =
              __builtin_amdgcn_exp2f(kPre ? S[kt][8 * sp + j] : fmaf(S[kt][8 * sp + j], a.scale_log2, -m_run));
          psum += p;
          v[j] = static_cast<__bf16>(p);
        }
        pb[2 * kt + sp] = v;
      }
    l_run += psum;
    // keep the whole softmax in this phase: s_barrier orders memory only, and without this the
    // compiler sinks the exp/cvt work across it into the MFMA phase that consumes P
    asm volatile("" ::"v"(pb[0]), "v"(pb[1]), "v"(pb[2]), "v"(pb[3]), "v"(l_run));
  };

  typedef std::integral_constant<int, 0> B0;
  typedef std::integral_constant<int, 1> B1;

  // kPersist, after the MFMA phase of tile t (in the wave's next VALU phase): t closed its block -> store
  // and zero O; t + 2 opens a block -> its Q, read by the next phase's Q K^T(t + 2)
  // buffer descriptors (SGPRs) + one VGPR byte offset per access, the d offsets as immediates: plain pointers
  // here had the compiler hoist 16 store and 8 load addresses out of the tile loop and spill (host-checked:
  // Lq * row stride fits 31 bits)
  const auto q_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)qp, (short)0, 0x7fffffff, 0x00020000);
  const auto o_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.o + b * a.o_sb + h * a.o_sh), (short)0, 0x7fffffff, 0x00020000);
  auto reload_q = [&](int t) __attribute__((always_inline)) {
    if ((t + 2) % ntk == 0 && t + 2 < ntiles) {
      const int row = min((qb + (t + 2) / ntk) * kQBlk + wave * kQRows + l31, a.Lq - 1);
      const int off = row * (int)a.q_sl * 2 + 16 * hl;
#pragma unroll
      for (int s = 0; s < 8; ++s)
        qf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(q_rsrc, off + 32 * s, 0, 0));
    }
  };
  auto block_boundary = [&](int t) __attribute__((always_inline)) {
    if ((t + 1) % ntk == 0) {
      const int row = (qb + t / ntk) * kQBlk + wave * kQRows + l31;
      const float inv = 1.f / wave_swap_sum(l_run);
      if (row < a.Lq) {
        const int off = row * (int)a.o_sl * 2 + 8 * hl;
#pragma unroll
        for (int db = 0; db < 4; ++db)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            u16x4 w;
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] = f2bf(o[db][4 * g + e] * inv);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, w), o_rsrc, off + 2 * (32 * db + 8 * g), 0, 0);
            __builtin_amdgcn_sched_barrier(0);  // one 4-value group at a time: no 64 live products
          }
      }
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
      l_run = 0.f;
    }
    reload_q(t);
  };

  // ---- prologue: K(0), V(0) -> buffer 0; K(1) -> buffer 1; S(0) for everyone, P(0) for A ----
  load_tile(0);
  if (group_b) write_k(B0{}); else write_v(B0{});
  if (group_b) {
    load_tile(1);
    write_k(B1{});
    load_tile(2);  // written in phase 0
  } else {
    load_tile(1);  // written in phase 1
  }
  __syncthreads();
  qk_mma(B0{});
  if constexpr (kPersist) {
    if (ntk == 1) reload_q(-1);  // one-tile blocks: Q of block 1 for Q K^T(1)
  }
  if (!group_b) softmax(0);
  __syncthreads();

  // one MFMA phase: QK^T of tile t+1 (if any) and P.V of tile t; t's parity picks the buffers
  // (the QK^T after the last tile reads a stale K buffer; its scores are never used).
  // MFMA j = 0..15: S[j&1] += K(rows 32(j&1)..) Q^T step j>>1 (one ds_read_b128 operand);
  // MFMA j = 16..31: O^T[d block (j-16)&3] += V^T P^T step (j-16)>>2 (two ds_read_b64_tr_b16).
  // The operand reads are inline asm issued four MFMAs ahead into a 5-deep register ring, each MFMA
  // preceded by a counted lgkmcnt wait that names its operand ("+v": no use before the data lands).
  // Nothing else touches LGKM in this phase (the barrier before it drained LDS and SMEM).
  auto mfma_phase = [&](auto PAR) __attribute__((always_inline)) {
    constexpr int par = decltype(PAR)::value;
    constexpr int kb = (par ^ 1) ? KB1 : 0;  // K(t+1)
    constexpr int vb = par ? kVBuf : 0;         // V(t), relative to V0
    // lab only (tools/lab/build.sh -DCP25_LAB_QK_HALF / -DCP25_LAB_PV_HALF, wrong results): drop half of the
    // QK^T (k-steps 4-7) or P.V (k-steps 2-3) MFMAs and their operand reads, the MFMA and LDS work an fp8 operand
    // (2x MFMA rate, half the bytes) would remove; the softmax VALU is unchanged
#ifndef CP25_LAB_QK_HALF
#define CP25_LAB_QK_HALF 0
#endif
#ifndef CP25_LAB_PV_HALF
#define CP25_LAB_PV_HALF 0
#endif
    constexpr auto lab_skip = [](int j) constexpr {
      return kF8 ? j < 16 : (CP25_LAB_QK_HALF && j >= 8 && j < 16) || (CP25_LAB_PV_HALF && j >= 24 && j < 32);
    };
    bf16x8 ring[5];
    auto issue = [&](auto JC) __attribute__((always_inline)) {
      constexpr int j = decltype(JC)::value;
      if constexpr (lab_skip(j)) {
      } else if constexpr (j < 16) {
        constexpr int off = kb + (j & 1) * 32 * KSTR + 32 * (j >> 1);
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ring[j % 5]) : "v"(k_rd_lds), "i"(off));
      } else if constexpr (j < 32) {
        constexpr int off = vb + 16 * ((j - 16) >> 2) * kVStride + 64 * ((j - 16) & 3);
        s16x4 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(v_rd_lds), "i"(off));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(v_rd_lds), "i"(off + 8 * kVStride));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        ring[j % 5] = __builtin_bit_cast(bf16x8, r);
      }
    };
    constexpr auto nreads = [=](int j) constexpr { return lab_skip(j) ? 0 : (j < 16 ? 1 : (j < 32 ? 2 : 0)); };
    // the MFMA-phase wave outranks its softmax partner in issue arbitration (+8% measured)
    __builtin_amdgcn_s_setprio(1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the counted waits below assume an empty LGKM queue
    if constexpr (kF8) {
      // QK^T(t+1) on fp8: 4 MFMAs, their 8 reads compiler-scheduled, done before the P.V ring starts
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
          S[kt] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(k_frag8(kb, kt, s), qf8[s],
                                                                 s == 0 ? (kF8 >= 2 ? sinit : zero16) : S[kt],
                                                                 0, 0, 0, 0, 0, 0);
      if constexpr (kF8 >= 2) {
        // P.V(t) on fp8: A = V^T (e4m3, cbsz 0), B = P^T (e5m2, blgp 1)
        constexpr int vbb = par ? kVBuf : 0;
#pragma unroll
        for (int db = 0; db < 4; ++db)
          o[db] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(v_frag8(vbb, db), pb8, o[db], 0, 1, 0, 0, 0, 0);
        if constexpr (kF8 == 3) lsum = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ones8, pb8, lsum, 0, 1, 0, 0, 0, 0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(0);
        return;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    static_for<4>(issue);
    static_for<32>([&](auto JC) __attribute__((always_inline)) {
      constexpr int j = decltype(JC)::value;
      issue(std::integral_constant<int, j + 4>{});
      constexpr int pending = nreads(j + 1) + nreads(j + 2) + nreads(j + 3) + nreads(j + 4);
      asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(ring[j % 5]) : "i"(pending));
      if constexpr (lab_skip(j)) {
      } else if constexpr (j < 16) {
        S[j & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ring[j % 5], qf[j >> 1], j < 2 ? zero16 : S[j & 1], 0, 0, 0);
      } else {
        o[(j - 16) & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ring[j % 5], pb[(j - 16) >> 2], o[(j - 16) & 3], 0, 0, 0);
      }
    });
    __builtin_amdgcn_s_setprio(0);
  };
  if (!group_b) {
    // group A: phase 2t MFMA, phase 2t+1 softmax(t+1) + V(t+1) staging
    auto step = [&](auto PAR, int t) __attribute__((always_inline)) {
      constexpr int par = decltype(PAR)::value;
      mfma_phase(PAR);
      ATTN_STAMP(t, 0);
      __syncthreads();
      ATTN_STAMP(t, 1);
      if (t + 1 < ntiles) {
        // the staged V(t+1) goes to LDS before the softmax: its LDS write drains under the VALU
        // (+0.9 % measured against writing after the softmax)
        write_v(std::integral_constant<int, par ^ 1>{});
        if constexpr (kPersist) block_boundary(t);
        softmax(t + 1);
        ATTN_STAMP(t, 5);
        load_tile(t + 2);
      } else if constexpr (kPersist) {
        block_boundary(t);
      }
      ATTN_STAMP(t, 2);
      __syncthreads();
      ATTN_STAMP(t, 3);
    };
    // pairs of tiles (constexpr buffer parity), then the odd last tile: one loop exit
    for (int t = 0; t + 1 < ntiles; t += 2) {
      step(B0{}, t);
      step(B1{}, t + 1);
    }
    if (ntiles & 1) step(B0{}, ntiles - 1);
  } else {
    // group B: phase 2t softmax(t) + K(t+2) staging, phase 2t+1 MFMA
    auto step = [&](auto PAR, int t) __attribute__((always_inline)) {
      if (t + 2 < ntiles) write_k(PAR);  // LDS write first, drains under the softmax VALU
      softmax(t);
      ATTN_STAMP(t, 4);
      if (t + 2 < ntiles) load_tile(t + 3);
      ATTN_STAMP(t, 0);
      __syncthreads();
      ATTN_STAMP(t, 1);
      mfma_phase(PAR);
      ATTN_STAMP(t, 2);
      __syncthreads();
      ATTN_STAMP(t, 3);
      if constexpr (kPersist) block_boundary(t);
    };
    // pairs of tiles (constexpr buffer parity), then the odd last tile: one loop exit
    for (int t = 0; t + 1 < ntiles; t += 2) {
      step(B0{}, t);
      step(B1{}, t + 1);
    }
    if (ntiles & 1) step(B0{}, ntiles - 1);
  }

  if constexpr (kPersist) return;  // every block was stored at its boundary
  // ---- epilogue: O = O^T / l, bf16, row q, d = 32db + 8g + 4hl + (0..3) ----
  const float l_tot = kF8 == 3 ? lsum[0] : wave_swap_sum(l_run);
  const float inv = kF8 >= 2 ? fmaxf(a.v_amax[bh], 0x1p-100f) * (1.f / 448.f) / l_tot : 1.f / l_tot;
  if (a.nsplit > 1) {
    // partial O of this key range (fp32, normalised by its own sum) + its log2-sum-exp2; merged by
    // attn_merge_splits
    if (q_row < a.Lq) {
      const int64_t row = ((int64_t)(split * a.B + b) * a.H + h) * a.Lq + q_row;
      float* op = a.o_part + row * kD;
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 w;
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = o[db][4 * g + e] * inv;
          *reinterpret_cast<f32x4*>(op + 32 * db + 8 * g + 4 * hl) = w;
        }
      if (hl == 0) a.lse_part[row] = m_run + __log2f(l_tot);
    }
    return;
  }
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

// ------------------------------------------------------------------------------------------------
// One wave per SIMD ("1w"): a workgroup = 4 waves = 256 query rows of one (b, h); each wave owns 64
// rows as two 32-row q-blocks and the whole register file (launch bound 1 wave/SIMD; O and Q live in
// the accumulator file, the softmax in the arch VGPRs). The wave is software-pipelined over 32-key
// half tiles with a lag of two on P.V: sub-step i issues
//     QK^T(i+1)  (16 MFMAs, K rows from LDS)   and   P.V(i-1)  (16 MFMAs, V rows from LDS, P(i-1))
// none of which depends on this sub-step's VALU, and runs the softmax of half i (S(i), computed in
// sub-step i-1, -> P(i)) in their issue gaps: 32 scores per lane = 32 exp + 32 fma + 32 add + 16
// packs, 3.5 VALU per MFMA gap with one transcendental each (MI355X_MICROARCH: <= 5 fillers per
// 32x32x16 gap hide behind the matrix pipe); there is no partner wave to arbitrate with.
// Same MFMA fragments as attn_fwd_d128 (swapped S^T = K Q^T, O^T = V^T P^T, V^T by transposed LDS
// reads of row-major V) and the same padded LDS rows; bounded-shift / prescaled softmax only (the
// DiT's forms; the online-max form stays on attn_fwd_d128).
// One loop iteration t = two sub-steps (halves 2t, 2t+1) and one barrier; it reads K(t), K(t+1),
// V(t-1), V(t) and writes K(t+2), V(t+1) into a 3-deep LDS ring (K(j) / V(j) in slot j % 3: K(t+2)
// overwrites K(t-1), V(t+1) overwrites V(t-2), both last read in iteration t-1). Register-staged by all
// four waves one iteration ahead: the iteration opens with the LDS writes of the tiles loaded in the
// previous iteration, then issues the loads of K(t+3) / V(t+2), which stay in flight across the
// barrier (the global latency is covered by a whole iteration).
constexpr int kThreads1w = 256;

// S^T MFMAs of attn_fwd_1w as inline asm: the scores must land in arch VGPRs (the softmax reads them
// with VALU; the builtin puts them in the accumulator file and copies them back, 32 v_accvgpr_read per
// half tile), with the Q operand held in the accumulator file. hipcc pads nothing inside an asm
// string, so the string carries its own wait states: `s_nop 1` ahead of the MFMA covers a
// v_accvgpr_write of the Q operand (or a VALU write of K) just before it (VALU -> MFMA operand: 2
// states). MFMA D -> VALU read: every consumer of these results is issued >= 3 MFMAs later (the next
// sub-step's softmax) or behind the explicit s_nops after the prologue.
__device__ __forceinline__ void mfma_s_init(f32x16& d, const bf16x8& k, const bf16x8& q) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(k), "a"(q));
}
__device__ __forceinline__ void mfma_s_acc(f32x16& d, const bf16x8& k, const bf16x8& q) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(k), "a"(q));
}
constexpr int kLds1w = 3 * kKBuf + 3 * kVBuf;  // 113664
// kDma (CP25_ATTN_KERNEL=1d): K/V tiles land in LDS by LDS-DMA (buffer_load ... lds) instead of the register
// staging: no staging VGPRs, no ds_write. The DMA image is lane-linear, so the rows are unpadded (256 B) and
// XOR-swizzled on the source side: K 16-B chunk c of row r at c ^ (r & 15) (the 16 rows a ds_read_b128 lane
// group reads at one column land on 16 distinct slots), V 64-B block b of row r at b ^ (r & 3) (the 4 rows of a
// transposed-read group on 4 distinct quarters). A 4-deep ring per operand lets the DMA run two tiles ahead.
constexpr int kDRow = 2 * kD;                    // 256 B
constexpr int kDTile = kKBlk * kDRow;            // 16 KiB
constexpr int kLds1wDma = 8 * kDTile;            // K slots 0-3, V slots 0-3: 128 KiB

// one 16-B-per-lane LDS-DMA piece, as inline asm: with the builtin the compiler cannot tell the DMA's LDS writes
// from the ring slots being read and puts an s_waitcnt vmcnt(0) before every LDS read of the loop (draining the
// two-tile-deep DMA queue); the kernel's own counted vmcnt + barrier order the slots instead
__device__ __forceinline__ void dma16_lds(__amdgpu_buffer_rsrc_t rsrc, __attribute__((address_space(3))) void* dst,
                                          int voffset) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)dst);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(m0), "v"(voffset), "s"(rsrc)
               : "memory", "m0");
}

template <int kKind, bool kPre, bool kDma = false>
__global__ void __launch_bounds__(kThreads1w, 1) attn_fwd_1w(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[kDma ? kLds1wDma : kLds1w];

  const int nwg = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int qblk = tile % a.nqb, bhs = tile / a.nqb;
  const int split = bhs % a.nsplit, bh = bhs / a.nsplit;
  const int b = bh / a.H, h = bh % a.H;
  const int key0 = split * a.tps * kKBlk;
  const int Lk = min(a.Lk - key0, a.tps * kKBlk);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l31 = lane & 31;
  const int hl = lane >> 5;

  const unsigned short* qp = a.q + b * a.q_sb + h * a.q_sh;
  const unsigned short* kp = a.k + b * a.k_sb + h * a.k_sh + (int64_t)key0 * a.k_sl;
  const unsigned short* vp = a.v + b * a.v_sb + h * a.v_sh + (int64_t)key0 * a.v_sl;

  // ---- Q fragments of the wave's two q-blocks, and each row's fixed softmax shift ----
  bf16x8 qf[2][8];
  float m_sh[2];
  int q_row[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    q_row[j] = qblk * kQBlk + wave * 64 + 32 * j + l31;
    const int qc = q_row[j] < a.Lq ? q_row[j] : a.Lq - 1;
    const unsigned short* src = qp + (int64_t)qc * a.q_sl + 8 * hl;
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[j][s] = *reinterpret_cast<const bf16x8*>(src + 16 * s);
    if constexpr (kPre) {
      m_sh[j] = 0.f;
    } else {
      float qq = 0.f;
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = static_cast<float>(qf[j][s][e]);
          qq = fmaf(x, x, qq);
        }
      qq = wave_swap_sum(qq);
      m_sh[j] = fmaxf(sqrtf(qq) * a.kbound * a.scale_log2 - kTop, 0.f);
    }
  }

  f32x16 o[4][2];
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[d][j][r] = 0.f;
  float l_run[2] = {0.f, 0.f};

  const int ntiles = (Lk + kKBlk - 1) / kKBlk;

  // ---- staging: all 256 threads, 4 x 16 B of a 64-row tile each: rows tid/16 + 16 i ----
  const int srow = tid >> 4, sch = tid & 15;
  const int stk_off = (int)(srow * a.k_sl * 2) + sch * 16, stk_step = (int)(16 * a.k_sl * 2);
  const int stv_off = (int)(srow * a.v_sl * 2) + sch * 16, stv_step = (int)(16 * a.v_sl * 2);
  u32x4 stk[4], stv[4];  // staged K(t+3) / V(t+2), in flight across the iteration's barrier (register mode)
  // DMA mode: wave w fills 1-KiB pieces w + 4u (u < 4) of a tile = rows 4 (w + 4u) + lane / 16; lane l writes
  // physical chunk l % 16 of its row, so it loads the logical chunk that the swizzle puts there
  int dk_src[4], dv_src[4];
  if constexpr (kDma) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = 4 * (wave + 4 * u) + (lane >> 4);
      const int pc = lane & 15;
      const int lck = pc ^ (row & 15);
      const int lcv = (((pc >> 2) ^ (row & 3)) << 2) | (pc & 3);
      dk_src[u] = row * (int)(a.k_sl * 2) + lck * 16;
      dv_src[u] = row * (int)(a.v_sl * 2) + lcv * 16;
    }
  }
  // tile t of K (kv = 0) or V (kv = 1); tiles past the end read as zeros (empty descriptor)
  auto tile_rsrc = [&](int kv, int t) __attribute__((always_inline)) {
    const int64_t sl = kv ? a.v_sl : a.k_sl;
    const unsigned short* base = kv ? vp : kp;
    const int rows = max(min(Lk - t * kKBlk, kKBlk), 0);
    const int nbytes = __builtin_amdgcn_readfirstlane(rows * (int)(sl * 2) - (rows > 0 ? (int)(sl * 2) - 2 * kD : 0));
    const uintptr_t addr = (uintptr_t)(base + (int64_t)min(t, ntiles - 1) * kKBlk * sl);
    const uintptr_t ua = ((uintptr_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(addr >> 32)) << 32) |
                         (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)addr);
    return __builtin_amdgcn_make_buffer_rsrc((void*)ua, (short)0, nbytes, 0x00020000);
  };
  auto load_tile = [&](int kv, int t, u32x4* st) __attribute__((always_inline)) {
    const int64_t sl = kv ? a.v_sl : a.k_sl;
    const unsigned short* base = kv ? vp : kp;
    // rows of tile t inside [0, Lk) (0 past the end), branch-free: the descriptor's range check
    // zero-fills the rest
    const int rows = max(min(Lk - t * kKBlk, kKBlk), 0);
    const int nbytes = __builtin_amdgcn_readfirstlane(rows * (int)(sl * 2) - (rows > 0 ? (int)(sl * 2) - 2 * kD : 0));
    // wave-uniform by construction; readfirstlane lets the compiler see it (no waterfall loops, T20)
    const uintptr_t addr = (uintptr_t)(base + (int64_t)min(t, ntiles - 1) * kKBlk * sl);
    const uintptr_t ua = ((uintptr_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(addr >> 32)) << 32) |
                         (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)addr);
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)ua, (short)0, nbytes, 0x00020000);
    const int off = kv ? stv_off : stk_off, step = kv ? stv_step : stk_step;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      st[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off + i * step, 0, 0));
  };
  // LDS slot bases (bytes): K slot j at j * kKBuf, V slot j at 3 kKBuf + j * kVBuf
  const int k_wr = srow * kKStride + sch * 16;
  const int v_wr = 3 * kKBuf + srow * kVStride + sch * 16;
  auto write_k = [&](int slot, const u32x4* st) __attribute__((always_inline)) {
    char* dst = smem + k_wr + slot * kKBuf;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<u32x4*>(dst + 16 * i * kKStride) = st[i];
  };
  auto write_v = [&](int slot, const u32x4* st) __attribute__((always_inline)) {
    char* dst = smem + v_wr + slot * kVBuf;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<u32x4*>(dst + 16 * i * kVStride) = st[i];
  };

  // per-lane LDS read offsets (the slot base is added once per iteration, the rest is immediate)
  constexpr int VSTR = kDma ? kDRow : kVStride;
  constexpr int KBUF = kDma ? kDTile : kKBuf, VBUF = kDma ? kDTile : kVBuf;
  constexpr int VBASE = kDma ? 4 * kDTile : 3 * kKBuf;  // V slot 0
  constexpr int NSLOT = kDma ? 4 : 3;
  const int grp = lane >> 4, gi = lane & 15;
  const int tq = gi >> 2, tp = gi & 3;
  // register mode: padded rows, everything but the slot an immediate; DMA mode: the swizzled chunk / block
  // depends on the lane, so the row base is per lane and the chunk / block offset is added per read
  const int k_rd = kDma ? l31 * kDRow : l31 * kKStride + 16 * hl;
  const int v_rd = kDma ? VBASE + (4 * (grp >> 1) + tq) * kDRow + 32 * (grp & 1) + 8 * tp
                        : 3 * kKBuf + (4 * (grp >> 1) + tq) * kVStride + 32 * (grp & 1) + 8 * tp;
  const int kx = l31 & 15;  // DMA mode: K row swizzle (row & 15 = l31 & 15 for every 32-row half)

  auto k_frag = [&](const char* kb, int kt, int s) __attribute__((always_inline)) {
    if constexpr (kDma) return *reinterpret_cast<const bf16x8*>(kb + kt * 32 * kDRow + 16 * ((2 * s + hl) ^ kx));
    else return *reinterpret_cast<const bf16x8*>(kb + kt * 32 * kKStride + 32 * s);
  };
  // V^T fragment of k-step ks (16 keys) and d-block db: two transposed 4x16-bit reads
  auto v_frag = [&](const char* vb, int ks, int db) __attribute__((always_inline)) {
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const int off = kDma ? 16 * ks * kDRow + 64 * (db ^ tq) : 16 * ks * kVStride + 64 * db;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds_char_ptr)(vb + off));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds_char_ptr)(vb + off + 8 * VSTR));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  };
  // DMA mode: the four pieces of this wave for tile t of K (kv 0) or V (kv 1) into a slot
  auto dma_piece = [&](const __amdgpu_buffer_rsrc_t& rs, int kv, int slot, int u, int t) __attribute__((always_inline)) {
    char* dst = smem + (kv ? VBASE : 0) + slot * kDTile + (wave + 4 * u) * 1024;
#ifdef CP25_ATTN_DMA_GLOBAL
    // lab (bench shape only: Lk % 64 == 0): global_load_lds with per-lane addresses instead of the buffer form
    const char* src = (const char*)(kv ? vp : kp) + (int64_t)min(t, ntiles - 1) * kKBlk * (kv ? a.v_sl : a.k_sl) * 2 +
                      (kv ? dv_src[u] : dk_src[u]);
    const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)dst);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" : : "s"(m0), "v"(src) : "memory", "m0");
    (void)rs;
#else
    (void)t;
    dma16_lds(rs, (__attribute__((address_space(3))) void*)dst, kv ? dv_src[u] : dk_src[u]);
#endif
  };

  f32x16 S[2][2];     // [half parity][q-block]: S^T of a 32-key half tile
  bf16x8 P[2][2][2];  // [half parity][q-block][k-step]: P^T of a half tile as P.V B operands
  const bf16x8 zero8 = {};

  // ---- prologue: K(0), K(1), V(0) -> slots 0, 1, 0; V slot 2 zeroed (V(-1) of the P.V(-1) of
  // sub-step 0, with P = 0); S(0) = QK^T(half 0) ----
  if constexpr (kDma) {
    // K(0), K(1), V(0) -> slots 0, 1, 0; V slot 3 (V(-1)) zeroed; K(2), V(1) in flight into slots 2, 1
    {
      const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int i = 0; i < 4; ++i) *reinterpret_cast<u32x4*>(smem + VBASE + 3 * kDTile + (tid + 256 * i) * 16) = z;
    }
    const auto rk0 = tile_rsrc(0, 0), rk1 = tile_rsrc(0, 1), rv0 = tile_rsrc(1, 0);
    const auto rk2 = tile_rsrc(0, 2), rv1 = tile_rsrc(1, 1);
#pragma unroll
    for (int u = 0; u < 4; ++u) dma_piece(rk0, 0, 0, u, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) dma_piece(rk1, 0, 1, u, 1);
#pragma unroll
    for (int u = 0; u < 4; ++u) dma_piece(rv0, 1, 0, u, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) dma_piece(rk2, 0, 2, u, 2);
#pragma unroll
    for (int u = 0; u < 4; ++u) dma_piece(rv1, 1, 1, u, 1);
    asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  } else {
    load_tile(0, 0, stk);
    write_k(0, stk);
    load_tile(0, 1, stk);
    write_k(1, stk);
    load_tile(1, 0, stv);
    write_v(0, stv);
    {
      const u32x4 z = {0u, 0u, 0u, 0u};
      const u32x4 zs[4] = {z, z, z, z};
      write_v(2, zs);
    }
    load_tile(0, 2, stk);  // written at the top of iteration 0
    load_tile(1, 1, stv);
    __syncthreads();
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const bf16x8 kf = k_frag(smem + k_rd, 0, s);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (s == 0) mfma_s_init(S[0][j], kf, qf[j][s]);
      else mfma_s_acc(S[0][j], kf, qf[j][s]);
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");  // S(0) -> the first softmax reads
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) P[1][j][sp] = zero8;

  // one sub-step: half i = 2t + SUB. QK^T(i+1) from K rows kq (32-row half kt_q) -> S[SUB^1];
  // softmax S[SUB] -> P[SUB]; P.V(i-1) from V half vh of the rows at vb with P[SUB^1]
  // LDS operands carried from one sub-step into the next: the first four K fragments and the first
  // two V fragments of a sub-step are read during the previous one (its groups 4..7), so no sub-step
  // opens on an LDS latency; every tile they read was written before the previous barrier
  bf16x8 ck[4], cv[2];
  auto sub_step = [&](auto SUBC, auto MASKC, int i, const char* kq, int kt_q, const char* vb, int vh,
                      const char* kq_n, int kt_n, const char* vb_n, int vh_n,
                      auto&& stage) __attribute__((always_inline)) {
    constexpr int c = decltype(SUBC)::value;  // parity of half i
    constexpr int n = c ^ 1;
    if (decltype(MASKC)::value && 32 * (i + 1) > Lk) {  // last tile only: keys >= Lk get -inf scores
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (key >= Lk) S[c][j][r] = -INFINITY;
        }
    }
    float psum[2] = {0.f, 0.f};
    // LDS operands: K fragments four groups ahead, V fragments two groups ahead, the first ones carried
    bf16x8 kfr[8], vfr[8];
#pragma unroll
    for (int g = 0; g < 4; ++g) kfr[g] = ck[g];
    vfr[0] = cv[0];
    vfr[1] = cv[1];
    __builtin_amdgcn_sched_barrier(0);
    // the issue stream, fixed by sched_barrier(0) fences: per group g, four (MFMA, VALU slice) pairs;
    // slice m handles score e = m of the group's four (fma, exp, row-sum add; a bf16 pack per pair)
    static_for<8>([&](auto GC) __attribute__((always_inline)) {
      constexpr int g = decltype(GC)::value;
      constexpr int pk = g >> 1, jj = pk & 1, sp = pk >> 1, hf = g & 1;
      float pv[4];
      static_for<4>([&](auto MC) __attribute__((always_inline)) {
        constexpr int m = decltype(MC)::value;
        if constexpr (m < 2) {  // QK^T(i+1), d-step g, q-block m
          if constexpr (g == 0) mfma_s_init(S[n][m], kfr[g], qf[m][g]);
          else mfma_s_acc(S[n][m], kfr[g], qf[m][g]);
        } else {  // P.V(i-1): k-step g >> 2 of the half, d-block g & 3, q-block m - 2
          o[g & 3][m - 2] =
              __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfr[g], P[n][m - 2][g >> 2], o[g & 3][m - 2], 0, 0, 0);
        }
        if constexpr (m == 0 && g + 2 < 8) vfr[g + 2] = v_frag(vb, 2 * vh + ((g + 2) >> 2), (g + 2) & 3);
        if constexpr (m == 1 && g < 4) kfr[g + 4] = k_frag(kq, kt_q, g + 4);
        if constexpr (m == 1 && g >= 4) ck[g - 4] = k_frag(kq_n, kt_n, g - 4);  // next sub-step's
        if constexpr (m == 3 && g >= 6) cv[g - 6] = v_frag(vb_n, 2 * vh_n, g - 6);
        if constexpr (m == 2 && g < 4) stage(g);  // one staged 16-B piece per group, in the MFMA shadow
        // softmax of half i: score e = m of pack (q-block jj, k-step sp), half hf
        const float sv = S[c][jj][8 * sp + 4 * hf + m];
        pv[m] = __builtin_amdgcn_exp2f(kPre ? sv : fmaf(sv, a.scale_log2, -m_sh[jj]));
        psum[jj] += pv[m];
        if constexpr (m & 1) {
          P[c][jj][sp][4 * hf + m - 1] = static_cast<__bf16>(pv[m - 1]);
          P[c][jj][sp][4 * hf + m] = static_cast<__bf16>(pv[m]);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    });
    l_run[0] += psum[0];
    l_run[1] += psum[1];
  };

  // iteration t: two sub-steps, stage K(t+2) and V(t+1), one barrier; only the last tile can be
  // ragged, so the main loop carries no masking (one basic block for the scheduler)
  auto iteration = [&](auto MASKC, int t, int slot) __attribute__((always_inline)) {
    // slot = t % NSLOT; s1 = (t+1) % NSLOT, sp = (t-1) % NSLOT (= (t+2) % 3 in register mode)
    const int s1 = slot == NSLOT - 1 ? 0 : slot + 1, s2 = slot == 0 ? NSLOT - 1 : slot - 1;
    const char* k_cur = smem + k_rd + slot * KBUF;
    const char* k_nxt = smem + k_rd + s1 * KBUF;
    const char* v_prv = smem + v_rd + s2 * VBUF;
    const char* v_cur = smem + v_rd + slot * VBUF;
    if constexpr (kDma) {
      // K(t+3) -> slot (t+3) % 4 = s2 (K(t-1), last read in iteration t-1), V(t+2) -> slot (t+2) % 4 (V(t-2))
      const int sk3 = s2, sv2 = s1 == NSLOT - 1 ? 0 : s1 + 1;
      const auto rk = tile_rsrc(0, t + 3);
      const auto rv = tile_rsrc(1, t + 2);
      sub_step(std::integral_constant<int, 0>{}, MASKC, 2 * t, k_cur, 1, v_prv, 1, k_nxt, 0, v_cur, 0,
               [&](int p) { dma_piece(rk, 0, sk3, p, t + 3); });
      sub_step(std::integral_constant<int, 1>{}, MASKC, 2 * t + 1, k_nxt, 0, v_cur, 0, k_nxt, 1, v_cur, 1,
               [&](int p) { dma_piece(rv, 1, sv2, p, t + 2); });
      // K(t+2) and V(t+1) (queued one iteration ago) land before the barrier; this iteration's 8 pieces fly on
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      return s1;
    }
    // staging, one 16-B piece per MFMA group, spread over the groups in the MFMA shadow (clustered at
    // the iteration start, the 8 loads + 8 LDS writes left the matrix pipe idle for ~500 cycles): piece
    // i of K(t+2) / V(t+1), loaded one iteration ago, goes to LDS, then piece i of K(t+3) / V(t+2) is
    // loaded into the same registers and flies across this iteration and its barrier
    const auto rk = tile_rsrc(0, t + 3);
    const auto rv = tile_rsrc(1, t + 2);
    char* const kdst = smem + k_wr + s2 * kKBuf;
    char* const vdst = smem + v_wr + s1 * kVBuf;
    // sub-step 0: QK^T(2t+1) = K(t) rows 32..63, softmax(2t), P.V(2t-1) = V(t-1) rows 32..63
    sub_step(std::integral_constant<int, 0>{}, MASKC, 2 * t, k_cur, 1, v_prv, 1, k_nxt, 0, v_cur, 0, [&](int p) {
      *reinterpret_cast<u32x4*>(kdst + 16 * p * kKStride) = stk[p];
      stk[p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, stk_off + p * stk_step, 0, 0));
    });
    // sub-step 1: QK^T(2t+2) = K(t+1) rows 0..31, softmax(2t+1), P.V(2t) = V(t) rows 0..31
    // (next: sub-step 0 of iteration t+1 = K(t+1) rows 32..63, V(t) rows 32..63)
    sub_step(std::integral_constant<int, 1>{}, MASKC, 2 * t + 1, k_nxt, 0, v_cur, 0, k_nxt, 1, v_cur, 1, [&](int p) {
      *reinterpret_cast<u32x4*>(vdst + 16 * p * kVStride) = stv[p];
      stv[p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rv, stv_off + p * stv_step, 0, 0));
    });
    __syncthreads();
    return s1;
  };
  // carried operands of iteration 0's sub-step 0: K(0) rows 32..63, V(-1) (the zeroed slot) rows 32..63
#pragma unroll
  for (int g = 0; g < 4; ++g) ck[g] = k_frag(smem + k_rd, 1, g);
  cv[0] = v_frag(smem + v_rd + (NSLOT - 1) * VBUF, 2, 0);
  cv[1] = v_frag(smem + v_rd + (NSLOT - 1) * VBUF, 2, 1);
  int slot = 0;  // t % 3
  for (int t = 0; t < ntiles - 1; ++t) slot = iteration(std::false_type{}, t, slot);
  iteration(std::true_type{}, ntiles - 1, slot);

  // ---- drain: P.V(2 ntiles - 1) = V(ntiles - 1) rows 32..63 with P[1] ----
  {
    const int sl = (ntiles - 1) % NSLOT;
    const char* vb = smem + v_rd + sl * VBUF;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const bf16x8 vf = v_frag(vb, 2 + (g >> 2), g & 3);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        o[g & 3][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, P[1][j][g >> 2], o[g & 3][j], 0, 0, 0);
    }
  }

  // ---- epilogue: O = O^T / l, row q, d = 32 db + 8 g + 4 hl + (0..3) ----
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float l_tot = wave_swap_sum(l_run[j]);
    // contract guard: norm bounds below the real norms can only show as an overflowed row sum
    // (moderate violations are exact by shift invariance): poison the row (NaN); never taken
    // under the contract
    const float inv = l_tot < 3.0e38f ? 1.f / l_tot : __uint_as_float(0x7fc00000u);
    if (q_row[j] >= a.Lq) continue;
    if (a.nsplit > 1) {
      const int64_t row = ((int64_t)(split * a.B + b) * a.H + h) * a.Lq + q_row[j];
      float* op = a.o_part + row * kD;
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 w;
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = o[db][j][4 * g + e] * inv;
          *reinterpret_cast<f32x4*>(op + 32 * db + 8 * g + 4 * hl) = w;
        }
      if (hl == 0) a.lse_part[row] = m_sh[j] + __log2f(l_tot);
    } else {
      unsigned short* op = a.o + b * a.o_sb + h * a.o_sh + (int64_t)q_row[j] * a.o_sl;
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          u16x4 w;
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = f2bf(o[db][j][4 * g + e] * inv);
          *reinterpret_cast<u16x4*>(op + 32 * db + 8 * g + 4 * hl) = w;
        }
    }
  }
}

// O[b, q, h, :] = sum_s w_s O_s / sum_s w_s with w_s = exp2(lse_s - max_s lse_s): the key-range
// partials of one (b, h, q) row combined exactly as the online softmax would have. One thread per
// 4 head-dim elements (32 threads per row); HBM-bound.
__global__ void __launch_bounds__(256) attn_merge_splits(const float* __restrict__ o_part,
                                                        const float* __restrict__ lse_part, unsigned short* o,
                                                        int nsplit, int B, int H, int Lq, int64_t o_sb,
                                                        int64_t o_sl, int64_t o_sh) {
  const int64_t rows = (int64_t)B * H * Lq;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = gid >> 5;
  if (row >= rows) return;
  const int d = (int)(gid & 31) * 4;
  float mx = -INFINITY;
  for (int s = 0; s < nsplit; ++s) mx = fmaxf(mx, lse_part[s * rows + row]);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float den = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float w = __builtin_amdgcn_exp2f(lse_part[s * rows + row] - mx);
    const f32x4 v = *reinterpret_cast<const f32x4*>(o_part + (s * rows + row) * kD + d);
    acc += w * v;
    den += w;
  }
  const float inv = 1.f / den;
  const int q = (int)(row % Lq);
  const int bh = (int)(row / Lq);
  const int b = bh / H, h = bh % H;
  u16x4 w;
#pragma unroll
  for (int e = 0; e < 4; ++e) w[e] = f2bf(acc[e] * inv);
  *reinterpret_cast<u16x4*>(o + b * o_sb + (int64_t)q * o_sl + h * o_sh + d) = w;
}

// ------------------------------------------------------------------------------------------------
// attn_fwd_m16: the bounded-shift / prescaled kernel on v_mfma_f32_16x16x32_bf16 (the default for those forms).
// Same workgroup (8 waves x 32 query rows of one (b, h)), the same ping-pong schedule, K/V staging and
// double-buffered LDS tiles as attn_fwd_d128; only the MFMA shape differs. Why: under sustained MFMA load the
// chip's clock is set by power, and on random data it holds a higher clock on the 16x16x32 shape than on
// 32x32x16 at equal cycles per FLOP (MI355X_MICROARCH "DVFS give-back" item 7: 1.12-1.15x in bare loops;
// cdna_hip_programming §5.4 rule 28), while the d128 kernel already runs at that 32x32x16 loop's rate.
// Fragments (lane l, g = l >> 4, c = l & 15), per wave and 64-key tile:
//   S^T = K Q^T: 4 key blocks kb x 2 query halves qh x 4 d-steps s = 32 MFMAs. A = K[16 kb + c][32 s + 8 g ..]
//     (one ds_read_b128, shared by both qh), B = Q[16 qh + c][32 s + 8 g ..] (32 VGPRs resident), C: lane holds
//     keys 16 kb + 4 g + i (i < 4) of query 16 qh + c: every lane owns two query rows and 16 keys of each.
//   O^T = V^T P^T: 8 d blocks db x 2 qh x 2 key steps ks = 32 MFMAs. B = P^T packed lane-locally from the two S
//     blocks kb = 2 ks, 2 ks + 1 (k slot 8 g + j <-> key 32 ks + 16 (j >> 2) + 4 g + (j & 3)); A = V^T in that
//     same key order: two ds_read_b64_tr_b16 (rows 32 ks + 4 g + q and 32 ks + 16 + 4 g + q, columns 16 db + 4 p
//     for lane 16 g + 4 q + p), shared by both qh.
// A query row's sum is spread over the 4 lane groups; with the fixed shift nothing needs it before the epilogue
// (one cross-group reduction per row). LDS rows of 288 B (256 + 32) for both K and V: a ds_read_b128 of the K
// fragment is serviced in the four 16-lane groups {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, ... (MI355X_MICROARCH
// §LDS), which mix rows c = 0..15 of lane groups g and g + 1; at 288 B the 16-B slot is (2 c + g + 4 s) mod 16,
// distinct within every such group (the d128 kernel's 272 B gives (c + g) mod 16: one 2-way conflict per group and
// read, measured 64 extra LDS cycles per wave and tile). The transposed V reads (two 32-lane halves, 8 rows x 32
// B each) land on 8 distinct 32-B bank groups.
constexpr int kKStride16 = 288;
constexpr int kVStride16 = 288;
#ifndef CP25_M16_AHEAD
#define CP25_M16_AHEAD 3
#endif
constexpr int kAhead = CP25_M16_AHEAD;  // MFMA phase: operand pairs read ahead of their MFMAs
#ifndef CP25_M16_SCHED
#define CP25_M16_SCHED 1
#endif
constexpr bool kM16Sched = CP25_M16_SCHED;
#ifndef CP25_M16_EARLY_LOAD
#define CP25_M16_EARLY_LOAD 0
#endif
constexpr bool kEarlyLoad = CP25_M16_EARLY_LOAD;  // K/V staging loads issued before the softmax instead of after
#ifndef CP25_M16_LSUM
#define CP25_M16_LSUM 1
#endif
// row sums by MFMA: lsum[qh] += ones^T P^T (one 16x16x32 MFMA per key step and query half, 4 per tile) instead of
// 32 v_add_f32 per tile in the softmax phase; the sum is then of the bf16 P the P.V MFMAs used, and it arrives
// complete in every lane (the MFMA reduces over the 4 lane groups)
constexpr bool kLsum = CP25_M16_LSUM;
#ifndef CP25_M16_PV_FIRST
#define CP25_M16_PV_FIRST 1
#endif
// MFMA phase order: P.V(t) before Q K^T(t+1), so P^T (16 VGPRs) is dead before S^T (32) is written and the two
// share registers (the other order keeps both live through the phase)
constexpr bool kPvFirst = CP25_M16_PV_FIRST;
#ifndef CP25_M16_LSUM_FIRST
#define CP25_M16_LSUM_FIRST 0
#endif
constexpr bool kLsumFirst = CP25_M16_LSUM_FIRST;  // row-sum MFMAs at the MFMA phase's start (else after the P.V pairs)
#ifndef CP25_M16_LSUM_SOFTMAX
#define CP25_M16_LSUM_SOFTMAX 0
#endif
constexpr bool kLsumSoftmax = CP25_M16_LSUM_SOFTMAX;  // row-sum MFMAs at the end of the softmax phase instead
#ifndef CP25_M16_PRE_B
#define CP25_M16_PRE_B 1
#endif
// group B issues its MFMA phase's first operand reads at the end of its softmax phase, before the barrier
constexpr bool kPreB = CP25_M16_PRE_B;
constexpr int kKBuf16 = kKBlk * kKStride16;        // 18432
constexpr int kVBuf16 = kKBlk * kVStride16;        // 18432
constexpr int kLds16 = 2 * kKBuf16 + 2 * kVBuf16;  // 73728
// kVt (cp25_attn_fwd_prescaled_vt): V arrives as cp25_cast_v_bf16t's V^T tiles ([128 d][64 p], 16 KiB contiguous),
// LDS rows of 160 B (128 + 32): the fragment read (row 16 db + c, 16-B chunk 4 ks + g) lands on slot
// (10 c + g + 4 ks) mod 16, distinct within every ds_read_b128 lane group
constexpr int kVtStride = 160;
constexpr int kVtBuf = kD * kVtStride;             // 20480
constexpr int kLds16t = 2 * kKBuf16 + 2 * kVtBuf;  // 77824

__device__ __forceinline__ float group4_sum(float x) {  // sum over the 4 lane groups of 16 (lanes c, c+16, c+32, c+48)
  x += __shfl_xor(x, 16);
  return x + __shfl_xor(x, 32);
}

template <int kKind, bool kPre, bool kVt = false>
__global__ void __launch_bounds__(kThreads, 2) attn_fwd_m16(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[kVt ? kLds16t : kLds16];
  constexpr int KB1 = kKBuf16, VB0 = 2 * kKBuf16;
  constexpr int VBUF = kVt ? kVtBuf : kVBuf16;  // V buffer 1, relative to VB0

  const int nwg = gridDim.x;
#ifdef CP25_LAB_NOREMAP  // lab: dispatch order = tile order (all XCDs on the same (b, h) at a time)
  const int tile = blockIdx.x;
  (void)nwg;
#else
  const int tile = xcd_remap(blockIdx.x, nwg);
#endif
  const int qb = tile % a.nqb;
  const int bhs = tile / a.nqb;
  const int split = bhs % a.nsplit, bh = bhs / a.nsplit;
  const int b = bh / a.H, h = bh % a.H;
  const int key0 = split * a.tps * kKBlk;
  const int Lk = min(a.Lk - key0, a.tps * kKBlk);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int c16 = lane & 15;
  const int g = lane >> 4;
  const bool group_b = __builtin_amdgcn_readfirstlane(tid) >= kThreads / 2;

  const unsigned short* qp = a.q + b * a.q_sb + h * a.q_sh;
  const unsigned short* kp = a.k + b * a.k_sb + h * a.k_sh + (int64_t)key0 * a.k_sl;
  const unsigned short* vp = kVt ? (const unsigned short*)((const char*)a.v + ((int64_t)bh * a.ntk_v + key0 / kKBlk) * 16384)
                                 : a.v + b * a.v_sb + h * a.v_sh + (int64_t)key0 * a.v_sl;

  // ---- Q fragments (B operand): Q[16 qh + c][32 s + 8 g .. +7] ----
  int q_row[2];
  bf16x8 qf[2][4];
#pragma unroll
  for (int qh = 0; qh < 2; ++qh) {
    q_row[qh] = qb * kQBlk + wave * kQRows + 16 * qh + c16;
    const unsigned short* src = qp + (int64_t)min(q_row[qh], a.Lq - 1) * a.q_sl + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[qh][s] = *reinterpret_cast<const bf16x8*>(src + 32 * s);
  }

  f32x4 o[8][2];
#pragma unroll
  for (int d = 0; d < 8; ++d)
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) o[d][qh] = f32x4{0.f, 0.f, 0.f, 0.f};
  float l_run[2] = {0.f, 0.f};
  f32x4 lsum[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  typedef short s16x8v __attribute__((ext_vector_type(8)));
  const bf16x8 ones8 = __builtin_bit_cast(bf16x8, s16x8v{0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80});
  float m_run[2] = {0.f, 0.f};
  if constexpr (!kPre) {  // bounded shift: m = max(|q_row| * kbound * scale_log2 - kTop, 0)
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      float qq = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = static_cast<float>(qf[qh][s][e]);
          qq = fmaf(x, x, qq);
        }
      m_run[qh] = fmaxf(sqrtf(group4_sum(qq)) * a.kbound * a.scale_log2 - kTop, 0.f);
    }
  }

  const int ntiles = (Lk + kKBlk - 1) / kKBlk;

  // staging (as attn_fwd_d128): a group's 256 threads own rows u/16 + 16 i, chunk u%16 of a 64 x 128 tile
  // (kVt, group A: rows u/8 + 32 i, chunk u%8 of the 128 x 64 V^T tile, 16 KiB contiguous)
  const int u = tid & (kThreads / 2 - 1);
  const bool vt_stage = kVt && !group_b;
  const int srow = vt_stage ? u >> 3 : u >> 4, sch = vt_stage ? u & 7 : u & 15;
  const int64_t sl = group_b ? a.k_sl : (kVt ? 64 : a.v_sl);
  const char* sbase = group_b ? (const char*)kp : (const char*)vp;
  const int st_off = (int)(srow * sl * 2) + sch * 16, st_step = (int)((vt_stage ? 32 : 16) * sl * 2);
  u32x4 st[4];
  auto load_tile = [&](int t) __attribute__((always_inline)) {
    const int rows = min(Lk - t * kKBlk, kKBlk);
    const int nbytes = vt_stage ? (rows > 0 ? 16384 : 0) : (rows > 0 ? (int)((rows - 1) * sl * 2) + 2 * kD : 0);
#ifdef CP25_LAB_TILE0  // lab only (wrong results): every tile re-reads key tile 0 (cache-resident K/V stream)
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)sbase, (short)0, nbytes, 0x00020000);
#else
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(sbase + (int64_t)t * (vt_stage ? 16384 : kKBlk * sl * 2)), (short)0, nbytes, 0x00020000);
#endif
#pragma unroll
    for (int i = 0; i < 4; ++i)
      st[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, st_off + i * st_step, 0, 0));
  };
  char* const k_wr = smem + srow * kKStride16 + sch * 16;
  char* const v_wr = smem + VB0 + srow * (kVt ? kVtStride : kVStride16) + sch * 16;
  auto write_k = [&](auto BUF) __attribute__((always_inline)) {
    constexpr int kb = decltype(BUF)::value ? KB1 : 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<u32x4*>(k_wr + kb + 16 * i * kKStride16) = st[i];
  };
  auto write_v = [&](auto BUF) __attribute__((always_inline)) {
    constexpr int vb = decltype(BUF)::value ? VBUF : 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<u32x4*>(v_wr + vb + (kVt ? 32 * i * kVtStride : 16 * i * kVStride16)) = st[i];
  };

  // per-lane LDS read bases; everything else is an immediate offset
  const char* const k_rd = smem + c16 * kKStride16 + 16 * g;  // + KB + 16 kb rows + 64 s bytes
  const char* const v_rd = kVt ? smem + VB0 + c16 * kVtStride + 16 * g  // + VB + 16 db rows + 64 ks bytes
                               : smem + VB0 + (4 * g + (c16 >> 2)) * kVStride16 + 8 * (c16 & 3);  // + VB + rows + 32 db
  const unsigned k_rd_lds = (unsigned)(uintptr_t)(lds_char_ptr)k_rd;
  const unsigned v_rd_lds = (unsigned)(uintptr_t)(lds_char_ptr)v_rd;

  const int ragged_tile = (Lk % kKBlk) != 0 ? Lk / kKBlk : -1;

  f32x4 S[4][2];   // S^T of the tile awaiting its softmax: [key block][query half]
  bf16x8 pb[2][2]; // P^T of the tile awaiting its P.V: [key step][query half]
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

  auto qk_mma = [&](auto BUF) __attribute__((always_inline)) {
    constexpr int kb = decltype(BUF)::value ? KB1 : 0;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(k_rd + kb + k4 * 16 * kKStride16 + 64 * s);
#pragma unroll
        for (int qh = 0; qh < 2; ++qh)
          S[k4][qh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qh][s], s == 0 ? zero4 : S[k4][qh], 0, 0, 0);
      }
  };
  auto softmax = [&](int t) __attribute__((always_inline)) {
    if (__builtin_expect(t == ragged_tile, 0)) {
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = t * kKBlk + 16 * k4 + 4 * g + i;
          if (key >= Lk) {
            S[k4][0][i] = -INFINITY;
            S[k4][1][i] = -INFINITY;
          }
        }
    }
    asm volatile("" : "+v"(S[0][0]), "+v"(S[0][1]), "+v"(S[1][0]), "+v"(S[1][1]), "+v"(S[2][0]), "+v"(S[2][1]),
                 "+v"(S[3][0]), "+v"(S[3][1]));
    // contract guard (as attn_fwd_d128): an overflowed row sum poisons the rows instead of a silent wrong answer
    if (__builtin_expect(__any(kLsum ? fmaxf(lsum[0][0], lsum[1][0]) > 3.0e38f : fmaxf(l_run[0], l_run[1]) > 3.0e38f), 0)) {
      const float nan = __uint_as_float(0x7fc00000u);
#pragma unroll
      for (int d = 0; d < 8; ++d) o[d][0] = o[d][1] = f32x4{nan, nan, nan, nan};
    }
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      float psum = 0.f;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float sv = S[2 * ks + (j >> 2)][qh][j & 3];
#ifdef CP25_LAB_NOEXP  // lab only (wrong results): no transcendental in the softmax phase
          const float p = sv;
#else
          const float p = __builtin_amdgcn_exp2f(kPre ? sv : fmaf(sv, a.scale_log2, -m_run[qh]));
#endif
          if constexpr (!kLsum) psum += p;
          v[j] = static_cast<__bf16>(p);
        }
        pb[ks][qh] = v;
      }
      if constexpr (!kLsum) l_run[qh] += psum;
    }
    asm volatile("" ::"v"(pb[0][0]), "v"(pb[0][1]), "v"(pb[1][0]), "v"(pb[1][1]), "v"(l_run[0]), "v"(l_run[1]));
    if constexpr (kLsum && kLsumSoftmax) {
      // the row-sum MFMAs in the softmax phase: they fill the partner wave's MFMA-pipe gaps (it waits on LDS
      // operands) instead of lengthening this wave's MFMA phase, the critical one
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) lsum[qh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones8, pb[ks][qh], lsum[qh], 0, 0, 0);
    }
  };

  typedef std::integral_constant<int, 0> B0;
  typedef std::integral_constant<int, 1> B1;

  // ---- prologue: K(0), V(0) -> buffer 0; K(1) -> buffer 1; S(0) for everyone, P(0) for A ----
  load_tile(0);
  if (group_b) write_k(B0{}); else write_v(B0{});
  if (group_b) {
    load_tile(1);
    write_k(B1{});
    load_tile(2);  // written in phase 0
  } else {
    load_tile(1);  // written in phase 1
  }
  __syncthreads();
  qk_mma(B0{});
  if (!group_b) softmax(0);
  __syncthreads();

  // one MFMA phase: Q K^T of tile t+1 and P.V of tile t (64 MFMAs of 16 cycles = the 32 of the d128 kernel).
  // Operand pair n (one fragment, two MFMAs, one per query half): n < 16 the K fragment (kb = n & 3, s = n >> 2),
  // n >= 16 the V^T fragment (db = (n - 16) & 7, ks = (n - 16) >> 3). Reads are inline asm issued kAhead pairs
  // ahead into a (kAhead + 1)-deep ring, each pair preceded by a counted lgkmcnt wait naming its operand.
  constexpr int kR = kAhead + 1;
  bf16x8 ring[kR];  // operand ring of the MFMA phase (group B may fill its head before the phase's barrier)
#ifdef CP25_LAB_NOLDS
#pragma unroll
  for (int i = 0; i < kR; ++i) ring[i] = qf[1][i & 3];
#endif
  auto issue_pair = [&](auto PAR, auto NC) __attribute__((always_inline)) {
      constexpr int par = decltype(PAR)::value;
      constexpr int kbuf = (par ^ 1) ? KB1 : 0;  // K(t+1)
      constexpr int vbuf = par ? VBUF : 0;       // V(t), relative to VB0
      constexpr int n = decltype(NC)::value;
#ifdef CP25_LAB_NOLDS  // lab only (wrong results): the MFMA phase reads no LDS (operands stay in the ring)
      if constexpr (true) {
      } else
#endif
      if constexpr (kPvFirst ? (n >= 16 && n < 32) : n < 16) {
        constexpr int m = kPvFirst ? n - 16 : n;
        constexpr int off = kbuf + (m & 3) * 16 * kKStride16 + 64 * (m >> 2);
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ring[n % kR]) : "v"(k_rd_lds), "i"(off));
      } else if constexpr (kVt && n < 32) {
        constexpr int m = kPvFirst ? n : n - 16;  // db = m & 7, ks = m >> 3
        constexpr int off = vbuf + 16 * (m & 7) * kVtStride + 64 * (m >> 3);
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ring[n % kR]) : "v"(v_rd_lds), "i"(off));
      } else if constexpr (n < 32) {
        constexpr int m = kPvFirst ? n : n - 16;
#ifdef CP25_LAB_VB128  // lab only (wrong results): one ds_read_b128 per V^T fragment instead of two transposed reads
        constexpr int offb = vbuf + 32 * (m >> 3) * kVStride16 + 32 * (m & 7) - VB0;
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ring[n % kR]) : "v"(k_rd_lds), "i"(VB0 + offb));
        return;
#endif
        constexpr int off = vbuf + 32 * (m >> 3) * kVStride16 + 32 * (m & 7);
        s16x4 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(v_rd_lds), "i"(off));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(v_rd_lds), "i"(off + 16 * kVStride16));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        ring[n % kR] = __builtin_bit_cast(bf16x8, r);
      }
  };
  // PRE: the first kAhead pairs were issued before the barrier that opens the phase (group B: its V(t) and K(t+1)
  // were written at least one barrier earlier, so it may read them while finishing its softmax phase)
  int probe_t = 0;  // lab probe: the tile of the running MFMA phase (read only by ATTN_STAMP under CP25_ATTN_PROBE)
  (void)probe_t;
  auto mfma_phase = [&](auto PAR, auto PRE) __attribute__((always_inline)) {
    auto issue = [&](auto NC) __attribute__((always_inline)) { issue_pair(PAR, NC); };
    constexpr auto nreads = [](int n) constexpr {
#ifdef CP25_LAB_NOLDS
      return 0 * n;
#endif
#ifdef CP25_LAB_VB128
      return n >= 32 ? 0 : 1;
#endif
      return n >= 32 ? 0 : ((kVt || (kPvFirst ? n >= 16 : n < 16)) ? 1 : 2);
    };
    __builtin_amdgcn_s_setprio(1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (!decltype(PRE)::value) static_for<kAhead>(issue);
    if constexpr (kLsum && !kLsumSoftmax && kLsumFirst) {
      // the row-sum MFMAs need no LDS operand: they cover the first reads' latency at the phase start
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) lsum[qh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones8, pb[ks][qh], lsum[qh], 0, 0, 0);
      if constexpr (kM16Sched) __builtin_amdgcn_sched_barrier(0);
    }
    static_for<32>([&](auto NC) __attribute__((always_inline)) {
      constexpr int n = decltype(NC)::value;
      issue(std::integral_constant<int, n + kAhead>{});
      constexpr int pending = [=]() constexpr {
        int p = 0;
        for (int i = 1; i <= kAhead; ++i) p += nreads(n + i);
        return p;
      }();
      asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(ring[n % kR]) : "i"(pending));
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) {
        if constexpr (kPvFirst ? n >= 16 : n < 16) {
          constexpr int m = kPvFirst ? n - 16 : n;
          S[m & 3][qh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[n % kR], qf[qh][m >> 2], m < 4 ? zero4 : S[m & 3][qh],
                                                                  0, 0, 0);
        } else {
          constexpr int m = kPvFirst ? n : n - 16;
          o[m & 7][qh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[n % kR], pb[m >> 3][qh], o[m & 7][qh], 0, 0, 0);
        }
      }
      // program order = issue order: read n + kAhead, wait, the pair's two MFMAs (the scheduler otherwise sinks
      // MFMAs below later reads and renames accumulators, which costs v_mov copies)
      if constexpr (kLsum && !kLsumSoftmax && !kLsumFirst && kPvFirst && n == 15) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int qh = 0; qh < 2; ++qh) lsum[qh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones8, pb[ks][qh], lsum[qh], 0, 0, 0);
      }
      if constexpr (kM16Sched) __builtin_amdgcn_sched_barrier(0);
#ifdef CP25_ATTN_PROBE
      // lab probe: inside the MFMA phase, after the first operand pair (6) and after the P.V half (7)
      if constexpr (n == 0) ATTN_STAMP(probe_t, 6);
      if constexpr (n == 15) ATTN_STAMP(probe_t, 7);
#endif
    });
    if constexpr (kLsum && !kLsumSoftmax && !kLsumFirst && !kPvFirst) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) lsum[qh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones8, pb[ks][qh], lsum[qh], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  if (!group_b) {
    // group A: phase 2t MFMA, phase 2t+1 softmax(t+1) + V(t+1) staging
    auto step = [&](auto PAR, int t) __attribute__((always_inline)) {
      constexpr int par = decltype(PAR)::value;
      probe_t = t;
      mfma_phase(PAR, std::false_type{});
      ATTN_STAMP(t, 0);
      __syncthreads();
      ATTN_STAMP(t, 1);
      if (t + 1 < ntiles) {
        write_v(std::integral_constant<int, par ^ 1>{});
        if constexpr (kEarlyLoad) load_tile(t + 2);  // the staging registers are free once written to LDS
        softmax(t + 1);
        ATTN_STAMP(t, 5);
        if constexpr (!kEarlyLoad) load_tile(t + 2);
      }
      ATTN_STAMP(t, 2);
      __syncthreads();
      ATTN_STAMP(t, 3);
    };
    for (int t = 0; t + 1 < ntiles; t += 2) {
      step(B0{}, t);
      step(B1{}, t + 1);
    }
    if (ntiles & 1) step(B0{}, ntiles - 1);
  } else {
    // group B: phase 2t softmax(t) + K(t+2) staging, phase 2t+1 MFMA
    auto step = [&](auto PAR, int t) __attribute__((always_inline)) {
      if (t + 2 < ntiles) write_k(PAR);
      if (kEarlyLoad && t + 2 < ntiles) load_tile(t + 3);
      softmax(t);
      ATTN_STAMP(t, 4);
      if (!kEarlyLoad && t + 2 < ntiles) load_tile(t + 3);
      if constexpr (kPreB) static_for<kAhead>([&](auto NC) __attribute__((always_inline)) { issue_pair(PAR, NC); });
      ATTN_STAMP(t, 0);
      __syncthreads();
      ATTN_STAMP(t, 1);
      probe_t = t;
      mfma_phase(PAR, std::integral_constant<bool, kPreB>{});
      ATTN_STAMP(t, 2);
      __syncthreads();
      ATTN_STAMP(t, 3);
    };
    for (int t = 0; t + 1 < ntiles; t += 2) {
      step(B0{}, t);
      step(B1{}, t + 1);
    }
    if (ntiles & 1) step(B0{}, ntiles - 1);
  }

  // ---- epilogue: lane holds O^T[16 db + 4 g + i][16 qh + c]: row q_row[qh], d = 16 db + 4 g + (0..3) ----
#pragma unroll
  for (int qh = 0; qh < 2; ++qh) {
    const float l_tot = kLsum ? lsum[qh][0] : group4_sum(l_run[qh]);
    const float inv = 1.f / l_tot;
    if (q_row[qh] >= a.Lq) continue;
    if (a.nsplit > 1) {
      const int64_t row = ((int64_t)(split * a.B + b) * a.H + h) * a.Lq + q_row[qh];
      float* op = a.o_part + row * kD + 4 * g;
#pragma unroll
      for (int db = 0; db < 8; ++db) {
        f32x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = o[db][qh][e] * inv;
        *reinterpret_cast<f32x4*>(op + 16 * db) = w;
      }
      if (g == 0) a.lse_part[row] = m_run[qh] + __log2f(l_tot);
    } else {
      unsigned short* op = a.o + b * a.o_sb + h * a.o_sh + (int64_t)q_row[qh] * a.o_sl + 4 * g;
#pragma unroll
      for (int db = 0; db < 8; ++db) {
        u16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = f2bf(o[db][qh][e] * inv);
        *reinterpret_cast<u16x4*>(op + 16 * db) = w;
      }
    }
  }
}

int g_num_cus = 0;

// the bounded / prescaled bf16 forms run on attn_fwd_m16 (16x16x32); CP25_ATTN_MFMA=32 selects attn_fwd_d128
// (32x32x16) instead. Same box, metric shape, prescaled: 143.3 / 143.6 ms vs 149.6 / 149.3 ms per launch
// (profiles/r2/attn_m16/). Read per launch (A/B runs and tests switch it in-process)
bool attn_m16() {
  const char* e = getenv("CP25_ATTN_MFMA");
  return !(e && e[0] == '3');
}

// which bounded/prescaled kernel runs: attn_fwd_d128 (two waves per SIMD, ping-pong; the default) or,
// with CP25_ATTN_KERNEL=1w, attn_fwd_1w (one wave per SIMD). Measured at the metric shape, prescaled
// form, same box: 1w 151.0 ms vs 2w 146.3 ms per launch (first version 172 vs 159.5;
// then the staging spread over the MFMA groups and carried LDS operands); 1w holds ~1.94 GHz with the
// MFMA pipe busy 62 % of cycles, 2w ~1.62 GHz at 78 %. Without any K/V staging the 1w loop runs
// 121-134 ms: what is left is hiding the global loads without a second wave. Read once.
// CP25_ATTN_KERNEL=1d: the one-wave-per-SIMD kernel with LDS-DMA staging (attn_fwd_1w<.., kDma>): 147.8 ms vs
// 2w 146.9 and register-staged 1w 151.2 (same box, prescaled, metric shape); PMC: 1.82 GHz at 69 % MFMA busy
// (2w: 1.62 GHz at 78 %), 50 GB of HBM reads per launch (2w: 27 GB). With the DMA as a compiler builtin the
// loop got an s_waitcnt vmcnt(0) before every LDS read and ran 430 ms.
int g_use_1w = -1;
int attn_variant() {  // 0: 2w, 1: 1w, 2: 1w + DMA staging
  if (g_use_1w < 0) {
    const char* e = getenv("CP25_ATTN_KERNEL");
    g_use_1w = (e && e[0] == '1') ? (e[1] == 'd' ? 2 : 1) : 0;
  }
  return g_use_1w;
}
bool use_1w() { return attn_variant() != 0; }

// CP25_XATTN_KERNEL=persist: the persistent short-KV form (opt-in: measured 3 % slower than one workgroup per
// query block at the DiT's cross-attention shape); read per launch (A/B runs and the
// bit-exactness test switch it in-process)
bool xattn_persistent() {
  const char* e = getenv("CP25_XATTN_KERNEL");
  return e && e[0] == 'p';
}

int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    g_num_cus = n;
  }
  return g_num_cus;
}

// Work-balance model for the key-range split: the kernel holds one workgroup per CU (252 VGPRs,
// 2 waves/SIMD), every workgroup's time is ~ its key tiles + a fixed ~44 tiles, and workgroups run
// in ceil(nwg / CUs) rounds; a split adds the fp32 partial write + merge traffic (~1 tile of time per
// 9 MB at HBM rate). The fixed cost is fitted to MI355X measurements (tools/bench_cp_chunks.py:
// B 2, H 16, Lq 13640, Lk 109120 ran 21.9 ms unsplit vs 23.0 ms at split 4; H 4: 6.24 vs 6.14 ms):
// shorter workgroups lose the lock-step K/V streaming through the XCD's L2 that long ones keep.
// Picks the split with the least modelled time.
int plan_split(int B, int H, int Lq, int Lk) {
  const int64_t nqb = cdiv(Lq, kQBlk), ntiles = cdiv(Lk, kKBlk);
  const int64_t nwg = nqb * B * H, cus = num_cus();
  int best = 1;
  double best_cost = 1e300;
  for (int s = 1; s <= 8 && s <= ntiles; ++s) {
    const int64_t tps = cdiv(ntiles, s);
    if (cdiv(ntiles, tps) != s) continue;  // every split must own at least one tile
    const double rounds = (double)cdiv(nwg * s, cus);
    double cost = rounds * (double)(tps + 44);
    if (s > 1) cost += (2.0 * s + 0.5) * (double)B * H * Lq * kD * 4 / 9.0e6;
    if (cost < best_cost * 0.995) { best_cost = cost; best = s; }
  }
  return best;
}

}  // namespace

#ifdef CP25_ATTN_PROBE
static unsigned long long* g_probe = nullptr;
static int g_probe_t0 = 0;
extern "C" void cp25_attn_probe_set(unsigned long long* probe, int t0) { g_probe = probe; g_probe_t0 = t0; }
#endif

static int attn_launch(const void* q, const void* k, const void* v, void* o, int B, int H, int Lq, int Lk, int D,
                       const int64_t* q_strides, const int64_t* k_strides, const int64_t* v_strides,
                       const int64_t* o_strides, float softmax_scale, float q_norm_bound, float k_norm_bound,
                       int n_split, void* workspace, size_t ws_bytes, hipStream_t stream, bool prescaled = false,
                       int fp8 = 0, const float* v_amax = nullptr, bool vt = false) {
  // vt: v is cp25_cast_v_bf16t's V^T tile layout (prescaled bf16 form on attn_fwd_m16 only; v_strides unused)
  if (vt && (fp8 || !prescaled)) return CP25_ERR_INVAL;
  // fp8: 1 = Q K^T on e4m3 q / k; 2 = also P.V on e5m2 P and the e4m3 v8t layout (v = v8t, v_strides unused)
  const bool fp8qk = fp8 >= 1;
  if (D != kD) return CP25_ERR_DTYPE;
  if (fp8qk && !prescaled) return CP25_ERR_INVAL;
  if (fp8 == 2 && (!v_amax || ((uintptr_t)v_amax & 3))) return CP25_ERR_INVAL;
  if (prescaled && !(q_norm_bound > 0.f && k_norm_bound > 0.f && (double)q_norm_bound * k_norm_bound <= (double)kTop))
    return CP25_ERR_INVAL;
  if (B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0) return CP25_ERR_INVAL;
  if (!q || !k || !v || !o) return CP25_ERR_INVAL;
  if (!(softmax_scale > 0.f) || !(q_norm_bound >= 0.f) || !(k_norm_bound >= 0.f) || q_norm_bound > 1e18f ||
      k_norm_bound > 1e18f)
    return CP25_ERR_INVAL;
  // rows must be 16-byte aligned for the vector loads / stores; head dim contiguous
  const int64_t* ss[4] = {q_strides, k_strides, v_strides, o_strides};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 3; ++j)
      if (!((fp8 == 2 || vt) && i == 2) && ss[i][j] % (fp8qk && i < 2 ? 16 : 8) != 0) return CP25_ERR_INVAL;  // 16 B rows
  // buffer_load offsets within a 64-key tile are 32-bit
  if ((int64_t)kKBlk * k_strides[1] * (fp8qk ? 1 : 2) >= (1ll << 31) ||
      (fp8 != 2 && !vt && (int64_t)kKBlk * v_strides[1] * 2 >= (1ll << 31)))
    return CP25_ERR_INVAL;
  if (k_strides[1] <= 0 || (fp8 != 2 && !vt && v_strides[1] <= 0)) return CP25_ERR_INVAL;
  if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) & 15) return CP25_ERR_INVAL;
  const int64_t ntiles = cdiv(Lk, kKBlk);
  if (n_split < 1 || n_split > ntiles) return CP25_ERR_INVAL;
  const int64_t tps = cdiv(ntiles, n_split);
  if (cdiv(ntiles, tps) != n_split) return CP25_ERR_INVAL;  // a split without keys
  const int64_t rows = (int64_t)B * H * Lq;
  if (n_split > 1) {
    if (!workspace || ((uintptr_t)workspace & 15) || ws_bytes < cp25_attn_workspace_bytes(B, H, Lq, n_split))
      return CP25_ERR_INVAL;
  }
  AttnArgs a;
  a.q = (const unsigned short*)q; a.k = (const unsigned short*)k; a.v = (const unsigned short*)v;
  a.o = (unsigned short*)o;
  a.q_sb = q_strides[0]; a.q_sl = q_strides[1]; a.q_sh = q_strides[2];
  a.k_sb = k_strides[0]; a.k_sl = k_strides[1]; a.k_sh = k_strides[2];
  a.v_sb = v_strides[0]; a.v_sl = v_strides[1]; a.v_sh = v_strides[2];
  a.o_sb = o_strides[0]; a.o_sl = o_strides[1]; a.o_sh = o_strides[2];
  a.B = B; a.H = H; a.Lq = Lq; a.Lk = Lk;
  a.nqb = (int)cdiv(Lq, kQBlk);
  a.nsplit = n_split;
  a.tps = (int)tps;
  a.nchunk = 1;
  a.ntk_v = (int)ntiles;
  a.v_amax = v_amax;
  // fp8 P.V: P = exp2(S - shift) <= 2^15 (e5m2 max 57344 = 2^15.8) for every score the norm bounds allow, with
  // the e4m3 rounding of q and k (each element within 2^-4 relative: |q8| |k8| <= 1.13 |q| |k|)
  a.s_init = -std::max(0.f, 1.13f * q_norm_bound * k_norm_bound - 15.f);
  a.o_part = n_split > 1 ? (float*)workspace : nullptr;
  a.lse_part = n_split > 1 ? (float*)workspace + (size_t)n_split * rows * kD : nullptr;
  a.scale_log2 = softmax_scale * 1.4426950408889634f;
  a.kbound = k_norm_bound;
  const bool fixed = q_norm_bound > 0.f && k_norm_bound > 0.f &&
                     (double)q_norm_bound * k_norm_bound * a.scale_log2 <= (double)kMaxBound;
#ifdef CP25_ATTN_PROBE
  a.probe = g_probe;
  a.probe_t0 = g_probe_t0;
#endif
  const int64_t nwg = (int64_t)a.nqb * B * H * n_split;
  if (nwg > 0x7fffffff) return CP25_ERR_INVAL;
  if (fp8 == 2) {
    // CP25_F8_EXP=exact: P by exp2 + cvt_pk_bf8 and fp32 row sums (the A/B reference of the integer form)
    const char* e = getenv("CP25_F8_EXP");
    const bool exact = e && e[0] == 'e';
    auto kernel = exact ? (Lk <= 4096 ? attn_fwd_d128<1, true, true, 2> : attn_fwd_d128<0, true, true, 2>)
                        : (Lk <= 4096 ? attn_fwd_d128<1, true, true, 3> : attn_fwd_d128<0, true, true, 3>);
    hipLaunchKernelGGL(kernel, dim3((unsigned)nwg), dim3(kThreads), 0, stream, a);
  } else if (fp8qk) {
    auto kernel = Lk <= 4096 ? attn_fwd_d128<1, true, true, 1> : attn_fwd_d128<0, true, true, 1>;
    hipLaunchKernelGGL(kernel, dim3((unsigned)nwg), dim3(kThreads), 0, stream, a);
  } else if ((prescaled || fixed) && use_1w()) {
    const bool dma = attn_variant() == 2;
    auto kernel = dma ? (prescaled ? (Lk <= 4096 ? attn_fwd_1w<1, true, true> : attn_fwd_1w<0, true, true>)
                                   : (Lk <= 4096 ? attn_fwd_1w<1, false, true> : attn_fwd_1w<0, false, true>))
                      : (prescaled ? (Lk <= 4096 ? attn_fwd_1w<1, true> : attn_fwd_1w<0, true>)
                                   : (Lk <= 4096 ? attn_fwd_1w<1, false> : attn_fwd_1w<0, false>));
    hipLaunchKernelGGL(kernel, dim3((unsigned)nwg), dim3(kThreads1w), 0, stream, a);
  } else if (prescaled && Lk <= 1024 && n_split == 1 && xattn_persistent() &&
             (int64_t)Lq * std::max(q_strides[1], o_strides[1]) * 2 < (1ll << 31)) {
    // short-KV (text cross-attention): one workgroup per CU over a contiguous run of query blocks
    const int64_t bhn = (int64_t)B * H;
    a.nchunk = (int)std::min<int64_t>(std::max<int64_t>(num_cus() / bhn, 1), a.nqb);
    if (bhn * a.nchunk > 0x7fffffff) return CP25_ERR_INVAL;
    hipLaunchKernelGGL((attn_fwd_d128<1, true, true, false, true>), dim3((unsigned)(bhn * a.nchunk)), dim3(kThreads), 0,
                       stream, a);
  } else if (vt) {
    auto kernel = Lk <= 4096 ? attn_fwd_m16<1, true, true> : attn_fwd_m16<0, true, true>;
    hipLaunchKernelGGL(kernel, dim3((unsigned)nwg), dim3(kThreads), 0, stream, a);
  } else if ((prescaled || fixed) && attn_m16()) {
    auto kernel = prescaled ? (Lk <= 4096 ? attn_fwd_m16<1, true> : attn_fwd_m16<0, true>)
                            : (Lk <= 4096 ? attn_fwd_m16<1, false> : attn_fwd_m16<0, false>);
    hipLaunchKernelGGL(kernel, dim3((unsigned)nwg), dim3(kThreads), 0, stream, a);
  } else {
    auto kernel = prescaled ? (Lk <= 4096 ? attn_fwd_d128<1, true, true> : attn_fwd_d128<0, true, true>)
                  : Lk <= 4096 ? (fixed ? attn_fwd_d128<1, true> : attn_fwd_d128<1, false>)
                               : (fixed ? attn_fwd_d128<0, true> : attn_fwd_d128<0, false>);
    hipLaunchKernelGGL(kernel, dim3((unsigned)nwg), dim3(kThreads), 0, stream, a);
  }
  CP25_LAUNCH_CHECK();
  if (n_split > 1) {
    const int64_t threads = rows * 32;
    hipLaunchKernelGGL(attn_merge_splits, dim3((unsigned)cdiv(threads, 256)), dim3(256), 0, stream, a.o_part,
                       a.lse_part, a.o, n_split, B, H, Lq, a.o_sb, a.o_sl, a.o_sh);
    CP25_LAUNCH_CHECK();
  }
  return CP25_OK;
}

extern "C" int cp25_attn_fwd_prescaled_fp8qk(const void* q8, const void* k8, const void* v, void* o, int B, int H,
                                             int Lq, int Lk, int D, const int64_t* q_strides,
                                             const int64_t* k_strides, const int64_t* v_strides,
                                             const int64_t* o_strides, float q_norm_bound, float k_norm_bound,
                                             int n_split, void* workspace, size_t ws_bytes, hipStream_t stream) {
  return attn_launch(q8, k8, v, o, B, H, Lq, Lk, D, q_strides, k_strides, v_strides, o_strides, 0.6931471805599453f,
                     q_norm_bound, k_norm_bound, n_split, workspace, ws_bytes, stream, true, 1);
}

extern "C" int cp25_attn_fwd_prescaled_fp8(const void* q8, const void* k8, const void* v8t, const float* v_amax,
                                           void* o, int B, int H, int Lq, int Lk, int D, const int64_t* q_strides,
                                           const int64_t* k_strides, const int64_t* o_strides, float q_norm_bound,
                                           float k_norm_bound, int n_split, void* workspace, size_t ws_bytes,
                                           hipStream_t stream) {
  const int64_t none[3] = {0, 0, 0};
  return attn_launch(q8, k8, v8t, o, B, H, Lq, Lk, D, q_strides, k_strides, none, o_strides, 0.6931471805599453f,
                     q_norm_bound, k_norm_bound, n_split, workspace, ws_bytes, stream, true, 2, v_amax);
}

extern "C" int cp25_attn_fwd_prescaled_vt(const void* q, const void* k, const void* vt, void* o, int B, int H, int Lq,
                                          int Lk, int D, const int64_t* q_strides, const int64_t* k_strides,
                                          const int64_t* o_strides, float q_norm_bound, float k_norm_bound, int n_split,
                                          void* workspace, size_t ws_bytes, hipStream_t stream) {
  const int64_t none[3] = {0, 0, 0};
  return attn_launch(q, k, vt, o, B, H, Lq, Lk, D, q_strides, k_strides, none, o_strides, 0.6931471805599453f,
                     q_norm_bound, k_norm_bound, n_split, workspace, ws_bytes, stream, true, 0, nullptr, true);
}

extern "C" size_t cp25_attn_workspace_bytes(int B, int H, int Lq, int n_split) {
  if (n_split <= 1 || B <= 0 || H <= 0 || Lq <= 0) return 0;
  return (size_t)n_split * B * H * Lq * (kD + 1) * sizeof(float);
}

extern "C" int cp25_attn_plan(int B, int H, int Lq, int Lk, int D) {
  if (D != kD) return CP25_ERR_DTYPE;
  if (B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0) return CP25_ERR_INVAL;
  return plan_split(B, H, Lq, Lk);
}

extern "C" int cp25_attn_fwd(const void* q, const void* k, const void* v, void* o, int B, int H, int Lq,
                             int Lk, int D, const int64_t* q_strides, const int64_t* k_strides,
                             const int64_t* v_strides, const int64_t* o_strides, float softmax_scale,
                             hipStream_t stream) {
  return attn_launch(q, k, v, o, B, H, Lq, Lk, D, q_strides, k_strides, v_strides, o_strides, softmax_scale, 0.f,
                     0.f, 1, nullptr, 0, stream);
}

extern "C" int cp25_attn_fwd_split(const void* q, const void* k, const void* v, void* o, int B, int H, int Lq,
                                   int Lk, int D, const int64_t* q_strides, const int64_t* k_strides,
                                   const int64_t* v_strides, const int64_t* o_strides, float softmax_scale,
                                   int n_split, void* workspace, size_t ws_bytes, hipStream_t stream) {
  return attn_launch(q, k, v, o, B, H, Lq, Lk, D, q_strides, k_strides, v_strides, o_strides, softmax_scale, 0.f,
                     0.f, n_split, workspace, ws_bytes, stream);
}

extern "C" int cp25_attn_fwd_bounded(const void* q, const void* k, const void* v, void* o, int B, int H, int Lq,
                                     int Lk, int D, const int64_t* q_strides, const int64_t* k_strides,
                                     const int64_t* v_strides, const int64_t* o_strides, float softmax_scale,
                                     float q_norm_bound, float k_norm_bound, int n_split, void* workspace,
                                     size_t ws_bytes, hipStream_t stream) {
  return attn_launch(q, k, v, o, B, H, Lq, Lk, D, q_strides, k_strides, v_strides, o_strides, softmax_scale,
                     q_norm_bound, k_norm_bound, n_split, workspace, ws_bytes, stream);
}

extern "C" int cp25_attn_fwd_prescaled(const void* q, const void* k, const void* v, void* o, int B, int H, int Lq,
                                       int Lk, int D, const int64_t* q_strides, const int64_t* k_strides,
                                       const int64_t* v_strides, const int64_t* o_strides, float q_norm_bound,
                                       float k_norm_bound, int n_split, void* workspace, size_t ws_bytes,
                                       hipStream_t stream) {
  return attn_launch(q, k, v, o, B, H, Lq, Lk, D, q_strides, k_strides, v_strides, o_strides, 0.6931471805599453f,
                     q_norm_bound, k_norm_bound, n_split, workspace, ws_bytes, stream, true);
}
