// Block projections of the DiT as bf16 MFMA GEMMs with fused epilogues (gfx950).
//
//   cp25_gemm_epi : C[M, N] = epi(A[M, K] W[N, K]^T), bf16 in / out, fp32 accumulation, replacing the
//                   block nn.Linear layers (no bias) of cosmos_predict2/_src/predict2/networks/
//                   minimal_v4_dit.py: Attention q/k/v/output projections (:354-363, :401-404, :432)
//                   and GPT2FeedForward layer1 / layer2 (:227-254). Epilogues:
//                     CP25_EPI_NONE : C = bf16(acc)
//                     CP25_EPI_GELU : C = bf16(gelu(bf16(acc))), exact-erf GELU on the bf16 layer1
//                                     output (:249-254: `x = self.layer1(x); x = self.activation(x)`),
//                                     the same arithmetic as cp25_gelu, so the MLP hidden never makes
//                                     the separate 2 x 3.6 GB GELU round trip.
//                     CP25_EPI_RES  : C = bf16(x + bf16(gate * bf16(acc))), the block's gated residual
//                                     (Block.forward :1204, :1237, :1246: x = x + gate * sublayer(x)) on the
//                                     output / cross-output / layer2 projections, with x and gate read by the
//                                     token-major row (tok, b) = (row / B, row % B) and the row's frame
//                                     (tok0 + tok) / hw; the next LN-mod then reads the new x once instead of x
//                                     and y (cp25_ln_mod with y = NULL).
//                     CP25_EPI_HNORM: C = bf16(bf16(RMSNorm_head(bf16(acc)) * w) * out_scale) per 128-column head,
//                                     the cross-attention q projection + its q_norm (:401-404, :411-419 without
//                                     RoPE) with cp25_head_rmsnorm_rope's partial sums, butterfly and roundings
//                                     (cp25_common.h hn_*): bit-identical to the GEMM followed by that kernel.
//                     CP25_EPI_QKV  : the fused q|k|v projection with the k columns' RMSNorm + 3D RoPE in the
//                                     epilogue (cp25_head_rmsnorm_rope's arithmetic again), q and v as bf16(acc).
//
// Design (MI355X, see DESIGN.md §3 "GEMM"): 256 x 256 output tile per 512-thread workgroup (one per
// CU), 8 waves as 2 (M) x 4 (N), each wave 128 x 64 with v_mfma_f32_16x16x32_bf16 (32 accumulators,
// the MFMA shape that holds the higher clock under load, MI355X_MICROARCH "DVFS" item 7); K in 64-deep
// tiles staged global -> LDS by LDS-DMA (one 1-KiB piece = 8 rows x 128 B per wave instruction). The LDS
// image is XOR-swizzled on the SOURCE side (16-B chunk c of row r lands at chunk c ^ ((r >> 1) & 7)),
// which makes every ds_read_b128 fragment read bank-conflict-free. Tiles are walked XCD-aware and
// grouped (8 row-tiles x all column tiles per group) so the workgroups resident on one XCD share
// their A and W tiles through that XCD's L2.
//   * gemm_nt_8ph (default, K/64 even): persistent, 8-phase schedule with counted vmcnt across raw barriers
//     and a pipelined tile seam (below).
//   * gemm_nt_kernel (odd K/64): the round-2 two-phase loop (vmcnt(0) + __syncthreads per K-tile), one workgroup
//     per tile. Both accumulate in the same order: bit-identical. Every output row is computed the same way
//     whatever M is (no split-K, fixed K order), so a context-parallel shard's rows equal the full run's bit for bit.
#include "cp25_common.h"

#include <algorithm>
#include <type_traits>

#pragma clang fp contract(off)

namespace {

constexpr int kBM = 256, kBN = 256, kBK = 64;
constexpr int kThreads = 512;
constexpr int kTileBytes = kBM * kBK * 2;       // 32 KiB per operand tile
constexpr int kStage = 2 * kTileBytes;          // A | W
constexpr int kLds = 2 * kStage;                // two stages: 128 KiB
constexpr int kGroupM = 8;

typedef __attribute__((address_space(3))) void* lds_void_ptr;

// compile-time loop: f(integral_constant<int, I>) for I = 0 .. N-1, in order
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

// one 16-B-per-lane buffer_load ... lds piece (a plain __device__ function: inside the kernel template the host pass
// drops the kernel's launch stub over this builtin)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, lds_void_ptr dst, int voffset, int soffset) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, 16, voffset, soffset, 0, 0);
}

__device__ __forceinline__ float gelu_exact(float a) { return gelu_erf(a); }  // = cp25_gelu (cp25_common.h)

// CP25_EPI_RES operands: output row r = token (r / B) batch entry (r % B); x element (tok, b, col) at
// tok * x_st + b * x_sb + col, gate element (b, frame, col) at b * g_sb + frame * g_st + col, frame = (tok0 + tok) / hw
// CP25_EPI_HNORM (the cross-attention's q projection, cp25_gemm_hnorm): per-head RMSNorm of the bf16 product with
// weight nw[128], eps, then x out_scale, the arithmetic of cp25_head_rmsnorm_rope without RoPE
struct ResEpi {
  const unsigned short* x; int64_t x_st, x_sb;
  const unsigned short* gate; int64_t g_sb, g_st;
  int B; int64_t tok0, hw;
  const unsigned short* nw; float n_eps, n_scale;
  // CP25_EPI_QKV: output columns [n_lo, n_hi) (the k projection) get nw's per-head RMSNorm and the rotate-half RoPE of
  // token row / B (rcos / rsin [tokens][64] fp32; nullptr: none), the others pass through
  const float* rcos; const float* rsin; int n_lo, n_hi;
};

// x + gate * y on 8 bf16 columns, two bf16 roundings (the reference's two torch ops, = cp25_ln_mod's residual)
__device__ __forceinline__ u32x4 res8(u32x4 y, u32x4 x, u32x4 g) {
  u32x4 o;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    unsigned r = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float yv = bf2f((unsigned short)(y[w] >> (16 * h)));
      const float xv = bf2f((unsigned short)(x[w] >> (16 * h)));
      const float gv = bf2f((unsigned short)(g[w] >> (16 * h)));
      r |= (unsigned)f2bf(rbf(xv + rbf(gv * yv))) << (16 * h);
    }
    o[w] = r;
  }
  return o;
}

template <int kEpi>
__global__ void __launch_bounds__(kThreads, 1)
gemm_nt_kernel(const unsigned short* __restrict__ A, int64_t lda, const unsigned short* __restrict__ W, int64_t ldw,
               unsigned short* __restrict__ C, int64_t ldc, int M, int N, int K, ResEpi re) {
  __shared__ __attribute__((aligned(16))) char smem[kLds];

  const int mt = (M + kBM - 1) / kBM, nt = N / kBN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int group = tile / (kGroupM * nt);
  const int first_m = group * kGroupM;
  const int gsize = min(mt - first_m, kGroupM);
  const int m_tile = first_m + (tile % (kGroupM * nt)) % gsize;
  const int n_tile = (tile % (kGroupM * nt)) / gsize;
  const int m0 = m_tile * kBM, n0 = n_tile * kBN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  // ---- LDS-DMA staging: wave w fills pieces 4w .. 4w+3 of each operand tile (piece = 8 rows) ----
  // lane l of a piece instruction writes LDS bytes [16 l, 16 l + 16) of the piece = row l / 8, chunk
  // position l % 8; it loads global chunk (l % 8) ^ swz(row) so the image is swizzled
  const int prow = lane >> 3, ppos = lane & 7;
  const unsigned short* a_src[4];
  const unsigned short* w_src[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = (wave * 4 + j) * 8 + prow;
    const int c = ppos ^ ((r >> 1) & 7);
    a_src[j] = A + (int64_t)min(m0 + r, M - 1) * lda + c * 8;
    w_src[j] = W + (int64_t)(n0 + r) * ldw + c * 8;
  }
  auto issue = [&](int kt, int buf) __attribute__((always_inline)) {
    char* sa = smem + buf * kStage;
    char* sw = sa + kTileBytes;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int piece = wave * 4 + j;
      __builtin_amdgcn_global_load_lds((const void*)(a_src[j] + kt * kBK), (lds_void_ptr)(sa + piece * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(w_src[j] + kt * kBK), (lds_void_ptr)(sw + piece * 1024), 16, 0, 0);
    }
  };

  // ---- fragment reads: lane (i = l % 16, g = l / 16) reads row i, k-chunk 4 s + g (16x16x32 layout) ----
  const int fr = lane & 15, fg = lane >> 4;
  int a_off[2], w_off[2];  // byte offsets within a tile for k-substep s (row base added per fragment)
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    // rows of a fragment start at a multiple of 16: swz(row) = (fr >> 1) & 7 for every fragment
    a_off[s] = fr * 128 + 16 * ((4 * s + fg) ^ ((fr >> 1) & 7));
    w_off[s] = a_off[s];
  }

  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = K / kBK;
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) issue(kt + 1, buf ^ 1);
    const char* sa = smem + buf * kStage + wm * 128 * 128;
    const char* sw = smem + buf * kStage + kTileBytes + wn * 64 * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[8], wf[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sa + i * 16 * 128 + a_off[s]);
#pragma unroll
      for (int j = 0; j < 4; ++j) wf[j] = *reinterpret_cast<const bf16x8*>(sw + j * 16 * 128 + w_off[s]);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], wf[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: bf16 (+ GELU) -> this wave's 128 x 64 tile in LDS -> 16-B row chunks to C ----
  // accumulator (i, j) register r: row 16 i + 4 (l / 16) + r, column 16 j + (l % 16)
  unsigned short* st = reinterpret_cast<unsigned short*>(smem + wave * 128 * 128);  // [128][64] bf16
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float y = rbf(acc[i][j][r]);
        if constexpr (kEpi == CP25_EPI_GELU) y = gelu_exact(y);
        st[(16 * i + 4 * fg + r) * 64 + 16 * j + fr] = f2bf(y);
      }
  // LDS accesses of one wave complete in order: this wave reads back only what it wrote
  const int row0 = m0 + wm * 128, col0 = n0 + wn * 64;
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int idx = it * 64 + lane;  // 128 rows x 8 chunks of 16 B
    const int r = idx >> 3, ch = idx & 7;
    if (row0 + r < M) {
      u32x4 v = *reinterpret_cast<const u32x4*>(st + r * 64 + ch * 8);
      if constexpr (kEpi == CP25_EPI_RES) {
        const int row = row0 + r, tok = row / re.B, b = row % re.B;
        const int64_t fr = (re.tok0 + tok) / re.hw;
        const u32x4 xv = *reinterpret_cast<const u32x4*>(re.x + tok * re.x_st + b * re.x_sb + col0 + ch * 8);
        const u32x4 gv = *reinterpret_cast<const u32x4*>(re.gate + b * re.g_sb + fr * re.g_st + col0 + ch * 8);
        v = res8(v, xv, gv);
      }
      *reinterpret_cast<u32x4*>(C + (int64_t)(row0 + r) * ldc + col0 + ch * 8) = v;
    }
  }
}


// ---------------------------------------------------------------------------------------------------------------
// 8-phase schedule (the default): the same tile, LDS image and MFMA shape, but the K loop is cut into four phases per
// 64-deep K-tile, one C quadrant (64 x 32 of the wave's 128 x 64) per phase, and the LDS-DMA stream runs 7 half-tiles
// ahead of the reads (a half-tile = 128 rows x 64 k of one operand, 16 KiB, 2 glds per thread):
//   * the two wave groups (wr = 0: waves 0-3, wr = 1: waves 4-7; one of each per SIMD) are staggered by one barrier,
//     so while one issues its quadrant's 16 MFMAs the other issues its LDS reads and its DMA piece;
//   * each phase: [fragment reads; one half-tile DMA] s_barrier [lgkmcnt(0); 16 MFMA at priority 1] s_barrier;
//   * quadrant order per K-tile (A half, B half): (0,0) reads B0 + A0, (0,1) reads B1, (1,1) reads A1, (1,0) reads
//     nothing (B0 kept in registers), so every read of K-tile t happens in its first three phases;
//   * DMA order per K-tile: B0, A0, B1, A1, issued for K-tile t+2 (same buffer as t) in phases 1-3 of t and phase 0 of
//     t+1: each half-tile is re-filled >= 2 phases after its last read (B0: 1 phase, its reads retired by the
//     lgkmcnt(8) before phase 0's first barrier);
//   * the only VM wait is a counted vmcnt(6) in phase 3 (3 half-tiles stay in flight across every barrier), which
//     retires K-tile t+1 before the barrier that precedes its first read; raw s_barrier (no __syncthreads, whose
//     fence would drain the DMA with vmcnt(0)), all LDS in one __shared__ array.
constexpr int kHalf = 128 * kBK * 2;  // 16 KiB
constexpr int kBuf8 = 4 * kHalf;      // A0 A1 B0 B1

// Persistent: one workgroup per CU walks tiles my_slot, my_slot + grid, ... (my_slot XCD-remapped). The tile
// seam is pipelined: after a tile's main loop its C tile is staged through the LDS into registers, then the NEXT
// tile's K-tiles 0 and 1 are queued (all 8 half-tiles) BEFORE this tile's 16 C stores, so every counted wait that
// follows can leave the stores in flight (the VM counter retires in order): vmcnt(24) retires the next K-tile 0,
// vmcnt(6 + 16) at phase 3 of K-tile 0 retires K-tile 1; by phase 3 of K-tile 1 the stores have had two K-tiles
// to drain. (Issued in the epilogue with a plain vmcnt(0) wait they cost 8-12 % at K = 2048.) A ragged last
// row-tile masks its stores, so the counts there fall back to vmcnt(0).
// CP25_EPI_RES: this thread's 16 x / gate chunks are loaded at the tile's end, once the accumulators are in the LDS
// (the VM queue is empty there: the last K-tile's phase 3 retired everything), land while C is read back, and are
// combined before the stores.
// (Round-2 A/B variants of this kernel -- skipped / nontemporal stores, the lab switches -- are in git history,
// DESIGN.md §3 "GEMM".)
// kES = 1 (cp25_gemm_fp8, config 5's fp8 option): A and W are OCP e4m3 bytes with a per-row scale of A and a per-row
// (output column) scale of W; a K-tile is 128 elements = the same 128-byte LDS rows, DMA pieces and fragment reads as
// the bf16 tile, and each (i, j) of a phase is ONE v_mfma_scale_f32_16x16x128_f8f6f4 over the lane's two 16-B chunks
// (k bytes 16 g .. and 64 + 16 g ..: the same k slots in A and B, which is all the sum needs) instead of two bf16
// MFMAs: twice the cycles each, half the count, twice the K -- 2x the bf16 rate. The epilogue multiplies each
// accumulator by a_scale[row] * w_scale[col] before the bf16 rounding (torch._scaled_mm's definition).
// GELU epilogue by table: the layer1 product is rounded to bf16 before the GELU, so GELU's bf16 result is a function of
// 16 input bits. gelu_tab holds bf16(gelu_erf(x)) for both signs and |x| in [2^-16, 8) (binary exponents 111 .. 129:
// 2 x 19 x 128 entries, 9.5 KiB of LDS, filled by each workgroup from the same gelu_erf): one LDS read per element
// instead of ~25 VALU operations (three of them transcendental), bit-identical; a wave with any input outside the
// table's range (|x| < 2^-16 or >= 8: rare) evaluates gelu_erf for those lanes.
constexpr int kGeluE0 = 111, kGeluNE = 19;
constexpr int kGeluTab = 2 * kGeluNE * 128;  // entries
__device__ __forceinline__ int gelu_tab_index(unsigned u) {  // u: bf16 bits; -1 outside the table
  // (exponent e, mantissa m) of one sign are the contiguous bit range [kGeluE0 128, (kGeluE0 + kGeluNE) 128): the
  // index is (u & 0x7fff) - kGeluE0 128 + sign kGeluNE 128 (3 VALU instead of 6 for the exponent / mantissa split)
  const unsigned m = (u & 0x7fffu) - (unsigned)(kGeluE0 * 128);
  return m < (unsigned)(kGeluNE * 128) ? (int)(m + (u >> 15) * (kGeluNE * 128)) : -1;
}

template <int kEpi, int kES = 2>
__global__ void __launch_bounds__(kThreads, 1)
gemm_nt_8ph(const unsigned short* __restrict__ A, int64_t lda, const unsigned short* __restrict__ W, int64_t ldw,
            unsigned short* __restrict__ C, int64_t ldc, int M, int N, int K, ResEpi re, const float* __restrict__ a_scale,
            const float* __restrict__ w_scale) {
  // fp8: 2 KiB past the K-tile buffers / C tile hold the tile's 256 row scales of A and 256 column scales of W
  __shared__ __attribute__((aligned(16)))
  char smem[2 * kBuf8 + (kES == 1 ? 2048 : 0) + (kEpi == CP25_EPI_GELU ? 2 * kGeluTab : 0)];
  static_assert(kES == 1 || kES == 2, "bf16 (2) or fp8 (1) operands");
  typedef int i32x8 __attribute__((ext_vector_type(8)));

  const int mt = (M + kBM - 1) / kBM, nt = N / kBN;
  const int n_tiles = mt * nt;
  const int nk = K * kES / (kBK * 2);  // 128-byte K-tiles
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int my_slot = xcd_remap(blockIdx.x, gridDim.x);

  // L2 grouping: 8 row tiles per group; 16 for the bf16 8192-wide MLP layer1 (same box, plain GEMMs at M = 218 240,
  // profiles/r4/gemm/group_ab.log: MLP1 5.48 vs 5.55 ms with 16, while QKV, MLP2 and the 2048-wide projections lose
  // 1.3-2 % with it). Tile order only: results bit-identical.
  const int gm = (kES == 2 && N >= 8192) ? 16 : kGroupM;
  auto tile_mn = [&](int tile, int& m0, int& n0) __attribute__((always_inline)) {
    const int group = tile / (gm * nt);
    const int first_m = group * gm;
    const int gsize = min(mt - first_m, gm);
    m0 = (first_m + (tile % (gm * nt)) % gsize) * kBM;
    n0 = ((tile % (gm * nt)) / gsize) * kBN;
  };
  // Tail plan (round 6): the F full rounds of the grid's P workgroups run whole tiles; the R tiles of the last, partial
  // round run as s row slices of 256 / s rows each when they fit in one round of slices: s = 4 if 4 R <= P, 2 if
  // 2 R <= P, else whole tiles. A slice is not s times cheaper: it still streams the whole W tile, runs every phase's
  // barriers and the whole epilogue; measured (tools/lab/gemm_tail/ab_tail.py, profiles/r6/gemm_tail/) a half slice
  // costs ~0.72 and a quarter ~0.55 of a tile (more with the GELU epilogue), so two rounds of slices never beat one
  // round of tiles. E.g. a CP = 8 rank's QKV (1296 tiles on 256 CUs: 16 left) runs 64 quarter slices, the whole
  // CFG batch's 2048-wide projections (856 tiles: 88 left) 176 halves. A slice is its parent tile with the rows outside it masked: the same LDS
  // image, DMA and phase schedule, MFMAs only for the slice's rows (a half tile: the first A half; a quarter: its first
  // wave row), so every output element is the same MFMA chain in the same K order as in a whole tile: rows stay
  // independent of M and of the plan (tests/test_gemm_gpu.py, test_configs_net_gpu.py CP = 8 rows).
  // The plan is recomputed at each tile seam from the launch's own values instead of being kept: the K loop sits at the
  // SGPR limit, and five more live scalars pushed the buffer descriptors into VGPRs (a readfirstlane waterfall per DMA
  // issue, +12 %). P is laundered so the compiler cannot hoist the plan out of the tile loop.
  auto plan = [&](int& FP, int& sd, int& nv) __attribute__((always_inline)) {
    int Pl = gridDim.x;
    asm volatile("" : "+s"(Pl));
    const int F = n_tiles / Pl, R = n_tiles - F * Pl;
    sd = 4 * R <= Pl ? 4 : (2 * R <= Pl ? 2 : 1);
    FP = F * Pl;
    nv = FP + R * sd;
  };
  // virtual tile v -> (m0, n0, rows of the slice); wave-uniform by construction and said so (readfirstlane), or the
  // buffer descriptors built from them count as divergent
  auto tile_at = [&](int v, int& m0, int& n0, int& rows) __attribute__((always_inline)) {
    int FP, sd, nv;
    plan(FP, sd, nv);
    if (v < FP) {
      tile_mn(v, m0, n0);
      rows = kBM;
    } else {
      const int j = v - FP;
      tile_mn(FP + j / sd, m0, n0);
      rows = kBM / sd;
      m0 += (j % sd) * rows;
    }
    m0 = __builtin_amdgcn_readfirstlane(m0);
    n0 = __builtin_amdgcn_readfirstlane(n0);
    rows = __builtin_amdgcn_readfirstlane(rows);
  };
  auto n_virtual = [&]() __attribute__((always_inline)) {
    int FP, sd, nv;
    plan(FP, sd, nv);
    return nv;
  };

  // ---- DMA (buffer_load ... lds): wave w fills pieces 2w, 2w+1 (8 rows each) of every half-tile; lane l -> row
  // l/8 of the piece, LDS chunk l%8, global chunk (l%8) ^ swz(row), swz(row) = (row >> 1) & 7. A's descriptor ends
  // at row M (a ragged last tile reads zeros there; those rows are not stored); W's per-wave / per-half row offsets
  // and the K advance ride in the scalar offset.
  const int prow = lane >> 3, ppos = lane & 7;
  int a_vo[2][2], w_vo[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = ppos ^ ((4 * j + (prow >> 1)) & 7);  // r = (2 wave + j) 8 + prow: (r >> 1) & 7 = (4 j + prow / 2) & 7
    w_vo[j] = prow * (int)ldw * kES + c * 16;
#pragma unroll
    for (int h = 0; h < 2; ++h) a_vo[h][j] = ((2 * wave + j) * 8 + h * 128 + prow) * (int)lda * kES + c * 16;
  }
  __amdgpu_buffer_rsrc_t a_rsrc, w_rsrc;
  // m_lim: the tile's row end, M or the end of its slice (rows past it read as zeros and are not stored). A slice of the
  // ragged last row tile may lie wholly past M (m_lim < m0): its descriptors then cover nothing (every clamp below
  // keeps its loads in bounds), its MFMAs run on zeros and it stores nothing.
  auto set_tile = [&](int m0, int n0, int m_lim) __attribute__((always_inline)) {
    // (the bound through readfirstlane: computed from the slice's row end it otherwise counts as divergent, and a
    // divergent descriptor turns every DMA issue of the K loop into a waterfall loop)
    const int a_bytes = __builtin_amdgcn_readfirstlane((int)((int64_t)max(0, min(m_lim - m0, kBM)) * lda * kES));
    a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)A + (int64_t)m0 * lda * kES), (short)0, a_bytes,
                                               0x00020000);
    w_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)W + (int64_t)n0 * ldw * kES), (short)0,
                                               (int)((int64_t)kBN * ldw * kES), 0x00020000);
  };
  // part 0: B half 0, 1: A half 0, 2: B half 1, 3: A half 1 (LDS: A0 @0, A1 @16K, B0 @32K, B1 @48K)
  auto issue = [&](int part, int kt, int buf) __attribute__((always_inline)) {
    const int h = part >> 1;
    const bool is_a = part & 1;
    char* dst = smem + buf * kBuf8 + (is_a ? 0 : 2 * kHalf) + h * kHalf + wave * 2048;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (is_a)
        dma16(a_rsrc, (lds_void_ptr)(dst + j * 1024), a_vo[h][j], kt * kBK * 2);
      else
        dma16(w_rsrc, (lds_void_ptr)(dst + j * 1024), w_vo[j], ((2 * wave + j) * 8 + h * 128) * (int)ldw * kES + kt * kBK * 2);
    }
  };
  // fp8: the tile's scales ride the DMA queue ahead of K-tile 0 (one dword per lane: waves 0-3 the 256 row scales of
  // A -- rows past M read 0 from the descriptor bound --, waves 4-7 the 256 column scales of W), so the epilogue
  // reads them from the LDS instead of paying a global-load round trip per tile. Retired with K-tile 0.
  auto issue_scales = [&](int m0, int n0, int m_lim) __attribute__((always_inline)) {
    if constexpr (kES == 1) {
      const bool is_a = wave < 4;
      const __amdgpu_buffer_rsrc_t s_rsrc = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(is_a ? a_scale + m0 : w_scale + n0), (short)0,
          __builtin_amdgcn_readfirstlane(is_a ? max(0, min(m_lim - m0, kBM)) * 4 : kBN * 4), 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(s_rsrc, (lds_void_ptr)(smem + 2 * kBuf8 + wave * 256), 4,
                                               ((wave & 3) * 64 + lane) * 4, 0, 0, 0);  // bound-checked offset
    }
  };
  auto issue_first_two = [&]() __attribute__((always_inline)) {  // K-tiles 0 and 1 of a tile (nk is even)
#pragma unroll
    for (int part = 0; part < 4; ++part) issue(part, 0, 0);
#pragma unroll
    for (int part = 0; part < 4; ++part) issue(part, 1, 1);
  };

  const int fr = lane & 15, fg = lane >> 4;
  const int frag0 = fr * 128 + 16 * ((0 + fg) ^ ((fr >> 1) & 7));  // k-substep 0
  const int frag1 = fr * 128 + 16 * ((4 + fg) ^ ((fr >> 1) & 7));  // k-substep 1
  const int a_row = wr * 64 * 128, b_row = wc * 32 * 128;

  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  f32x4_t acc[2][2][4][2];
  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
  bool stores_pending = false;  // this wave's previous-tile C stores are in flight, queued after K-tiles 0 and 1
  int t_rows = kBM;             // rows of the current tile (kBM, or a tail slice's; tile_at): read by the slice loop only

  auto phase = [&](auto qc, auto bc, int kt, auto slc) __attribute__((always_inline)) {
    constexpr int Q = decltype(qc)::value, BUF = decltype(bc)::value;
    constexpr bool kSlice = decltype(slc)::value;  // a tail row slice (tile_at): the K loop's second instance
    const char* sbuf = smem + BUF * kBuf8;
    if constexpr (Q == 0 || Q == 1) {
      const char* sb = sbuf + 2 * kHalf + Q * kHalf + b_row;
      auto& fb = Q == 0 ? fb0 : fb1;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        fb[j][0] = *reinterpret_cast<const bf16x8*>(sb + j * 16 * 128 + frag0);
        fb[j][1] = *reinterpret_cast<const bf16x8*>(sb + j * 16 * 128 + frag1);
      }
    }
    if constexpr (Q == 0) __builtin_amdgcn_sched_barrier(0);
    if constexpr (Q == 0 || Q == 2) {
      const char* sa = sbuf + (Q >> 1) * kHalf + a_row;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[i][0] = *reinterpret_cast<const bf16x8*>(sa + i * 16 * 128 + frag0);
        fa[i][1] = *reinterpret_cast<const bf16x8*>(sa + i * 16 * 128 + frag1);
      }
    }
    // DMA: K-tile kt + 1 part 3 (Q = 0; K-tile 1 was queued whole at the seam) or K-tile kt + 2 part Q - 1
    if constexpr (Q == 0) {
      if (kt > 0 && kt + 1 < nk) issue(3, kt + 1, BUF ^ 1);
    } else {
      if (kt + 2 < nk) issue(Q - 1, kt + 2, BUF);
    }
    if constexpr (Q == 0) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
    if constexpr (Q == 3) {
      // retire K-tile kt + 1; newer: K-tile kt + 2 parts 0-2 (6) and, at kt = 0, the previous tile's stores (16)
      if (kt + 2 >= nk)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (kt == 0 && stores_pending)
        asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    constexpr int mq = Q >> 1, nq = (Q == 1 || Q == 2);
    auto& fb = nq ? fb1 : fb0;
    // a row slice of the tail (tile_at): only the waves / A half holding its rows issue MFMAs (wave-uniform; whole
    // tiles run the K loop instance without this test)
    if (kSlice && !(mq == 0 && (t_rows == kBM / 2 || wr == 0))) {
    } else if constexpr (kES == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const u32x4 a0 = __builtin_bit_cast(u32x4, fa[i][0]), a1 = __builtin_bit_cast(u32x4, fa[i][1]);
          const u32x4 b0 = __builtin_bit_cast(u32x4, fb[j][0]), b1 = __builtin_bit_cast(u32x4, fb[j][1]);
          const i32x8 av = {(int)a0[0], (int)a0[1], (int)a0[2], (int)a0[3], (int)a1[0], (int)a1[1], (int)a1[2], (int)a1[3]};
          const i32x8 bv = {(int)b0[0], (int)b0[1], (int)b0[2], (int)b0[3], (int)b1[0], (int)b1[1], (int)b1[2], (int)b1[3]};
          acc[mq][nq][i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc[mq][nq][i][j], 0, 0, 0, 0, 0, 0);
        }
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[mq][nq][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], fb[j][s], acc[mq][nq][i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  int tile = my_slot;
  if (tile >= n_virtual()) return;
  u32x4 nwv = {0u, 0u, 0u, 0u};  // CP25_EPI_HNORM: this lane's 8 norm weights (columns 8 (ch & 15) .. of its head)
  if constexpr (kEpi == CP25_EPI_HNORM || kEpi == CP25_EPI_QKV) nwv = *reinterpret_cast<const u32x4*>(re.nw + (tid & 15) * 8);
#ifndef CP25_LAB_GELU_VALU
  if constexpr (kEpi == CP25_EPI_GELU) {  // the GELU table (visible after the prologue's barrier)
    unsigned short* tab = reinterpret_cast<unsigned short*>(smem + 2 * kBuf8);
    for (int i = tid; i < kGeluTab; i += kThreads) {
      const int r = i % (kGeluNE * 128);
      const unsigned u = (unsigned)(i / (kGeluNE * 128)) << 15 | (unsigned)(kGeluE0 + r / 128) << 7 | (unsigned)(r % 128);
      tab[i] = f2bf(gelu_exact(bf2f((unsigned short)u)));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
#endif
  int m0, n0;
  tile_at(tile, m0, n0, t_rows);
  set_tile(m0, n0, min(M, m0 + t_rows));
  issue_scales(m0, n0, min(M, m0 + t_rows));
  issue_first_two();
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // K-tile 0 (and the fp8 scales)
  __builtin_amdgcn_s_barrier();

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  while (true) {
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int nq = 0; nq < 2; ++nq)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[mq][nq][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger the second wave group by one barrier
    __builtin_amdgcn_sched_barrier(0);
    auto kloop = [&](auto slc) __attribute__((always_inline)) {
      for (int kt = 0; kt < nk; kt += 2) {
        phase(I0{}, I0{}, kt, slc);
        phase(I1{}, I0{}, kt, slc);
        phase(I2{}, I0{}, kt, slc);
        phase(I3{}, I0{}, kt, slc);
        phase(I0{}, I1{}, kt + 1, slc);
        phase(I1{}, I1{}, kt + 1, slc);
        phase(I2{}, I1{}, kt + 1, slc);
        phase(I3{}, I1{}, kt + 1, slc);
      }
    };
    if (t_rows == kBM)
      kloop(std::false_type{});
    else
      kloop(std::true_type{});
    int m_lim;
    {
      int m0_, n0_, rows_;
      tile_at(tile, m0_, n0_, rows_);
      m_lim = min(M, m0 + rows_);
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();
    // every wave's reads of this tile are done and no DMA is in flight: the LDS becomes the C tile. Raw barriers
    // (a __syncthreads() fence would also wait for C stores).
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    const int next = tile + gridDim.x;
    const bool has_next = next < n_virtual();
    // ---- C tile -> LDS [256][256] bf16 (row stride 512 B; 16-B chunk ch of row r at ch ^ sw(r), sw(r) =
    // 2 ((r >> 2) & 3) = 2 fg for this wave's rows, so the four row groups of a fragment write hit distinct banks).
    // Element (row, col): row = mq 128 + wr 64 + 16 i + 4 fg + r, col = nq 128 + wc 32 + 16 j + fr; the lane part
    // of the address has two values (j = 0, 1), the rest is an immediate. The bases are laundered per tile so the
    // compiler does not hoist them out of the tile loop (they would stay live across the K loop).
    // CP25_EPI_RES: this thread's 16 x chunks are requested first, into the registers the K loop's fragments held,
    // so their HBM latency runs under the staging below (requested after it, they waited out the whole latency at
    // the combine); the 16 gate chunks (L2-resident, one row per frame) follow the staging as before.
    // thread t owns rows m0 + 16 it + t / 32 (it = 0..15), 16-B chunk t % 32 of the C tile
    const int ch = tid & 31, r0 = tid >> 5;
    u32x4 xres[16], gres[16];
    if constexpr (kEpi == CP25_EPI_RES) {
      const int row_a = min(m0 + r0, m_lim - 1), tok_a = row_a / re.B, b = row_a % re.B, dtok = 16 / re.B;
      const unsigned short* xp = re.x + (int64_t)tok_a * re.x_st + b * re.x_sb + n0 + ch * 8;
      const int n_valid = (m_lim - 1 - row_a) / 16;  // rows row_a + 16 it, it <= n_valid, exist
      // the row offset is selected arithmetically (x 0 or 1): a selected POINTER made the compiler load the fallback
      // row first and branch around a second load behind a vmcnt(0) -- sixteen serialised HBM round trips per tile
#pragma unroll
      for (int it = 0; it < 16; ++it)
        xres[it] = *reinterpret_cast<const u32x4*>(xp + (int64_t)(it * dtok) * re.x_st * (int64_t)(it <= n_valid));
    }
    int ez = 0;
    asm volatile("" : "+v"(ez));
    unsigned short* const ct = reinterpret_cast<unsigned short*>(smem);
    unsigned short* stj[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
      stj[j] = ct + wr * 64 * 256 + (wc >> 1) * 64 + ez + 4 * fg * 256 +
               ((((wc & 1) * 4 + 2 * j + (fr >> 3)) ^ (2 * fg)) << 3) + (fr & 7);
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int nq = 0; nq < 2; ++nq)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float a = acc[mq][nq][i][j][r];
              if constexpr (kES == 1) {  // row mq 128 + wr 64 + 16 i + 4 fg + r, column nq 128 + wc 32 + 16 j + fr
                const float* sc = reinterpret_cast<const float*>(smem + 2 * kBuf8) + ez;
                const f32x4_t as = *reinterpret_cast<const f32x4_t*>(sc + mq * 128 + wr * 64 + 16 * i + 4 * fg);
                a = a * as[r] * sc[256 + nq * 128 + wc * 32 + 16 * j + fr];
              }
              stj[j][(mq * 128 + 16 * i + r) * 256 + nq * 128] = f2bf(rbf(a));  // (GELU: applied after the readback)
            }
    // (after the accumulators are in the LDS: their registers hold the gate chunks)
    if constexpr (kEpi == CP25_EPI_RES) {
      // row r0 + 16 it: token tok_a + it * (16 / B), batch entry b (16 % B == 0), frame by a running remainder that
      // wraps at most once per step (16 / B <= hw, host-checked): straight-line code. Rows past M (a ragged last
      // row-tile) read the thread's first valid row instead (their results are not stored).
      const int row_a = min(m0 + r0, m_lim - 1), tok_a = row_a / re.B, b = row_a % re.B, dtok = 16 / re.B;
      int64_t fr = (re.tok0 + tok_a) / re.hw, rem = (re.tok0 + tok_a) % re.hw;
      const unsigned short* gp = re.gate + b * re.g_sb + n0 + ch * 8;
      const int n_valid = (m_lim - 1 - row_a) / 16;  // rows row_a + 16 it, it <= n_valid, exist
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const bool ok = it <= n_valid;
        gres[it] = *reinterpret_cast<const u32x4*>(gp + fr * re.g_st * (int64_t)ok);
        rem += dtok;
        const bool wrap = rem >= re.hw;
        rem -= wrap ? re.hw : 0;
        fr += wrap ? 1 : 0;
      }
    }

    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // thread t reads rows 16 it + t / 32 (it = 0..15), 16-B chunk t % 32 (sw(row) depends on t only)
    const unsigned short* rd = ct + ez + r0 * 256 + ((ch ^ (((r0 >> 2) & 3) << 1)) << 3);
    u32x4 cv[16];
#pragma unroll
    for (int it = 0; it < 16; ++it) cv[it] = *reinterpret_cast<const u32x4*>(rd + it * 16 * 256);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // the LDS is free for the next tile's DMA
    if constexpr (kEpi == CP25_EPI_QKV) {
      if (n0 >= re.n_lo && n0 < re.n_hi) {  // a k tile (wave-uniform): RMSNorm + RoPE of its two heads per row
        // the tile's RoPE rows (tokens m0 / B .., 256 / B of them) come into the free LDS first (by LDS-DMA, one
        // exposed round trip; loaded per row into registers they were 16 serialised trips: +0.8 ms per launch)
        const int li = ch & 15, dlo = (li & 7) * 8;
        const float sgn = li < 8 ? -1.f : 1.f;
        const bool rope = re.rcos != nullptr;
        const int tok_lo = m0 / re.B;
        constexpr int kTabBytes = 65536;  // per table: up to 256 tokens x 64 fp32
        if (rope) {
          const int ntok = max(0, min(m_lim - 1, m0 + kBM - 1) / re.B - tok_lo + 1);
          const int nbytes = ntok * 256;
          const __amdgpu_buffer_rsrc_t c_rsrc = __builtin_amdgcn_make_buffer_rsrc(
              (void*)(re.rcos + (int64_t)tok_lo * 64), (short)0, nbytes, 0x00020000);
          const __amdgpu_buffer_rsrc_t s_rsrc = __builtin_amdgcn_make_buffer_rsrc(
              (void*)(re.rsin + (int64_t)tok_lo * 64), (short)0, nbytes, 0x00020000);
          for (int kb = wave; kb * 1024 < nbytes; kb += kThreads / 64) {  // 1 KiB (4 tokens) per wave instruction
            dma16(c_rsrc, (lds_void_ptr)(smem + kb * 1024), kb * 1024 + 16 * lane, 0);
            dma16(s_rsrc, (lds_void_ptr)(smem + kTabBytes + kb * 1024), kb * 1024 + 16 * lane, 0);
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
        const float* const tcos = reinterpret_cast<const float*>(smem);
        const float* const tsin = reinterpret_cast<const float*>(smem + kTabBytes);
#pragma unroll
        for (int it = 0; it < 16; ++it) {
          float v[8];
#pragma unroll
          for (int w2 = 0; w2 < 4; ++w2) {
            v[2 * w2] = bf2f((unsigned short)(cv[it][w2] & 0xffffu));
            v[2 * w2 + 1] = bf2f((unsigned short)(cv[it][w2] >> 16));
          }
          float ss = hn_sumsq8(v);
#pragma unroll
          for (int m = 8; m >= 1; m >>= 1) ss += __shfl_xor(ss, m, 16);
          const float rstd = hn_rstd(ss, re.n_eps);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            v[e] = hn_norm(v[e], rstd, bf2f((unsigned short)(nwv[e >> 1] >> (16 * (e & 1)))));
          if (rope) {
            const int tl = max(0, min(m0 + r0 + 16 * it, m_lim - 1) / re.B - tok_lo);
            const f32x4 c0 = *reinterpret_cast<const f32x4*>(tcos + tl * 64 + dlo);
            const f32x4 c1 = *reinterpret_cast<const f32x4*>(tcos + tl * 64 + dlo + 4);
            const f32x4 s0 = *reinterpret_cast<const f32x4*>(tsin + tl * 64 + dlo);
            const f32x4 s1 = *reinterpret_cast<const f32x4*>(tsin + tl * 64 + dlo + 4);
            float partner[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) partner[e] = __shfl_xor(v[e], 8, 16);
#pragma unroll
            for (int e = 0; e < 8; ++e)
              v[e] = hn_rope(v[e], partner[e], sgn, e < 4 ? c0[e & 3] : c1[e & 3], e < 4 ? s0[e & 3] : s1[e & 3]);
          }
          u32x4 o;
#pragma unroll
          for (int w2 = 0; w2 < 4; ++w2)
            o[w2] = (unsigned)f2bf(v[2 * w2] * re.n_scale) | ((unsigned)f2bf(v[2 * w2 + 1] * re.n_scale) << 16);
          cv[it] = o;
        }
        if (rope) {  // every wave's table reads are done before the next tile's DMA writes the LDS
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
      }
    }
    if constexpr (kEpi == CP25_EPI_RES) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the x / gate chunks (nothing else is in flight)
#pragma unroll
      for (int it = 0; it < 16; ++it)
        if (m0 + r0 + 16 * it < m_lim) cv[it] = res8(cv[it], xres[it], gres[it]);
    }

    unsigned short* crow = C + (int64_t)(m0 + r0) * ldc + n0 + ch * 8;
    const bool full = m0 + kBM <= m_lim;
    const int rows_left = m_lim - (m0 + r0);  // rows of C from this lane's first row (ragged last row-tile / slice)
    if (has_next) {
      tile = next;
      tile_at(tile, m0, n0, t_rows);
      set_tile(m0, n0, min(M, m0 + t_rows));
      issue_scales(m0, n0, min(M, m0 + t_rows));
      issue_first_two();
    }
    __builtin_amdgcn_sched_barrier(0);  // the DMAs are queued ahead of the stores (the counts above rely on it)
#ifdef CP25_LAB_GELU_VALU
    if constexpr (kEpi == CP25_EPI_GELU) {  // lab (tools/lab/gelu): gelu_erf on every element, no table
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        u32x4 o;
#pragma unroll
        for (int w2 = 0; w2 < 4; ++w2)
          o[w2] = (unsigned)f2bf(gelu_exact(bf2f((unsigned short)(cv[it][w2] & 0xffffu)))) |
                  ((unsigned)f2bf(gelu_exact(bf2f((unsigned short)(cv[it][w2] >> 16)))) << 16);
        cv[it] = o;
      }
    }
#else
    if constexpr (kEpi == CP25_EPI_GELU) {
      // the GELU on the read-back bf16 products, by table (its own LDS region, untouched by the DMA just queued, so the
      // lookups run under that DMA's latency instead of in the C staging before it); one wave-wide test per 8-element
      // chunk for an input outside the table, which then takes gelu_erf
      const unsigned short* tab = reinterpret_cast<const unsigned short*>(smem + 2 * kBuf8);
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        u32x4 o;
        bool miss = false;
#pragma unroll
        for (int w2 = 0; w2 < 4; ++w2) {
          const unsigned u0 = cv[it][w2] & 0xffffu, u1 = cv[it][w2] >> 16;
          const int t0 = gelu_tab_index(u0), t1 = gelu_tab_index(u1);
          miss |= (t0 | t1) < 0;
          o[w2] = (unsigned)tab[t0 < 0 ? 0 : t0] | ((unsigned)tab[t1 < 0 ? 0 : t1] << 16);
        }
        if (__builtin_expect(__any(miss), 0)) {
#pragma unroll
          for (int w2 = 0; w2 < 4; ++w2) {
            const unsigned u0 = cv[it][w2] & 0xffffu, u1 = cv[it][w2] >> 16;
            const unsigned g0 = gelu_tab_index(u0) < 0 ? f2bf(gelu_exact(bf2f((unsigned short)u0))) : (o[w2] & 0xffffu);
            const unsigned g1 = gelu_tab_index(u1) < 0 ? f2bf(gelu_exact(bf2f((unsigned short)u1))) : (o[w2] >> 16);
            o[w2] = g0 | (g1 << 16);
          }
        }
        cv[it] = o;
      }
    }
#endif
    if constexpr (kEpi == CP25_EPI_HNORM) {
      // lanes 16 h .. 16 h + 15 of a 32-lane row hold head h's 128 columns, lane li = ch & 15 the 8 columns 8 li ..:
      // cp25_head_rmsnorm_rope's item layout, so its butterfly over 16 lanes is this one (runs under the DMA above)
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        float v[8];
#pragma unroll
        for (int w2 = 0; w2 < 4; ++w2) {
          v[2 * w2] = bf2f((unsigned short)(cv[it][w2] & 0xffffu));
          v[2 * w2 + 1] = bf2f((unsigned short)(cv[it][w2] >> 16));
        }
        float ss = hn_sumsq8(v);
#pragma unroll
        for (int m = 8; m >= 1; m >>= 1) ss += __shfl_xor(ss, m, 16);
        const float rstd = hn_rstd(ss, re.n_eps);
        u32x4 o;
#pragma unroll
        for (int w2 = 0; w2 < 4; ++w2) {
          const float lo = hn_norm(v[2 * w2], rstd, bf2f((unsigned short)(nwv[w2] & 0xffffu)));
          const float hi = hn_norm(v[2 * w2 + 1], rstd, bf2f((unsigned short)(nwv[w2] >> 16)));
          o[w2] = (unsigned)f2bf(lo * re.n_scale) | ((unsigned)f2bf(hi * re.n_scale) << 16);
        }
        cv[it] = o;
      }
    }
    if (full) {
#pragma unroll
      for (int it = 0; it < 16; ++it) *reinterpret_cast<u32x4*>(crow + (int64_t)it * 16 * ldc) = cv[it];
    } else {
#pragma unroll
      for (int it = 0; it < 16; ++it)
        if (it * 16 < rows_left) *reinterpret_cast<u32x4*>(crow + (int64_t)it * 16 * ldc) = cv[it];
    }
    if (!has_next) return;
    // retire the next tile's K-tile 0: the stores (16, when all issued) and K-tile 1 (8) may stay in flight
    stores_pending = full;
    if (stores_pending)
      asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
}
}  // namespace

static int gemm_launch(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int M, int N,
                       int K, int epilogue, const ResEpi& re, hipStream_t stream) {
  if (!a || !w || !c || M <= 0 || N <= 0 || K <= 0) return CP25_ERR_INVAL;
  if (N % kBN != 0 || K % kBK != 0) return CP25_ERR_DTYPE;  // the tiles this kernel is built for
  if (lda < K || ldw < K || ldc < N || (lda % 8) || (ldw % 8) || (ldc % 8)) return CP25_ERR_INVAL;
  if (lda >= (1 << 22) || ldw >= (1 << 22)) return CP25_ERR_INVAL;  // 32-bit in-tile byte offsets
  if (((uintptr_t)a | (uintptr_t)w | (uintptr_t)c) & 15) return CP25_ERR_INVAL;
  if (epilogue != CP25_EPI_NONE && epilogue != CP25_EPI_GELU && epilogue != CP25_EPI_RES && epilogue != CP25_EPI_HNORM &&
      epilogue != CP25_EPI_QKV)
    return CP25_ERR_INVAL;
  if (epilogue == CP25_EPI_QKV) {
    if (re.B <= 0 || re.n_lo < 0 || re.n_hi > N || re.n_lo % kBN || re.n_hi % kBN || re.n_lo >= re.n_hi ||
        (!re.rcos) != (!re.rsin) || (((uintptr_t)re.rcos | (uintptr_t)re.rsin) & 15))
      return CP25_ERR_INVAL;
  }
  if (epilogue == CP25_EPI_HNORM || epilogue == CP25_EPI_QKV) {
    if (!re.nw || ((uintptr_t)re.nw & 15) || !(re.n_eps >= 0.f) || !(re.n_scale > 0.f)) return CP25_ERR_INVAL;
    if ((K / kBK) % 2 != 0) return CP25_ERR_DTYPE;  // the persistent kernel only (the caller runs the separate norm)
  }
  if (epilogue == CP25_EPI_RES) {
    if (!re.x || !re.gate || re.B <= 0 || 16 % re.B || re.hw < 16 / re.B || re.tok0 < 0 || (re.x_st % 8) || (re.x_sb % 8) ||
        (re.g_sb % 8) || (re.g_st % 8) || (((uintptr_t)re.x | (uintptr_t)re.gate) & 15))
      return CP25_ERR_INVAL;
    if ((int64_t)(M - 1) / re.B * re.x_st >= (1ll << 40)) return CP25_ERR_INVAL;
  }
  const int64_t nwg = (int64_t)((M + kBM - 1) / kBM) * (N / kBN);
  if (nwg > 0x7fffffff) return CP25_ERR_INVAL;
  const unsigned short* A = (const unsigned short*)a;
  const unsigned short* Wp = (const unsigned short*)w;
  unsigned short* Cp = (unsigned short*)c;
  const dim3 grid((unsigned)nwg), block(kThreads);
  static int n_cu[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return CP25_ERR_LAUNCH;
  if (!n_cu[dev] && hipDeviceGetAttribute(&n_cu[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return CP25_ERR_LAUNCH;
  const int cus = n_cu[dev] >= 8 ? n_cu[dev] & ~7 : n_cu[dev];
  // (up to 4 x the tiles: with fewer tiles than CUs the kernel's tail plan runs them as row slices)
  const dim3 pgrid((unsigned)std::min<int64_t>(4 * nwg, cus));
  if ((K / kBK) % 2 != 0) {
    switch (epilogue) {
      case CP25_EPI_GELU:
        hipLaunchKernelGGL(gemm_nt_kernel<CP25_EPI_GELU>, grid, block, 0, stream, A, lda, Wp, ldw, Cp, ldc, M, N, K, re);
        break;
      case CP25_EPI_RES:
        hipLaunchKernelGGL(gemm_nt_kernel<CP25_EPI_RES>, grid, block, 0, stream, A, lda, Wp, ldw, Cp, ldc, M, N, K, re);
        break;
      default:
        hipLaunchKernelGGL(gemm_nt_kernel<CP25_EPI_NONE>, grid, block, 0, stream, A, lda, Wp, ldw, Cp, ldc, M, N, K, re);
    }
  } else {
    switch (epilogue) {
      case CP25_EPI_GELU:
        hipLaunchKernelGGL((gemm_nt_8ph<CP25_EPI_GELU, 2>), pgrid, block, 0, stream, A, lda, Wp, ldw, Cp, ldc, M, N, K, re,
                           nullptr, nullptr);
        break;
      case CP25_EPI_RES:
        hipLaunchKernelGGL((gemm_nt_8ph<CP25_EPI_RES, 2>), pgrid, block, 0, stream, A, lda, Wp, ldw, Cp, ldc, M, N, K, re,
                           nullptr, nullptr);
        break;
      case CP25_EPI_HNORM:
        hipLaunchKernelGGL((gemm_nt_8ph<CP25_EPI_HNORM, 2>), pgrid, block, 0, stream, A, lda, Wp, ldw, Cp, ldc, M, N, K,
                           re, nullptr, nullptr);
        break;
      case CP25_EPI_QKV:
        hipLaunchKernelGGL((gemm_nt_8ph<CP25_EPI_QKV, 2>), pgrid, block, 0, stream, A, lda, Wp, ldw, Cp, ldc, M, N, K,
                           re, nullptr, nullptr);
        break;
      default:
        hipLaunchKernelGGL((gemm_nt_8ph<CP25_EPI_NONE, 2>), pgrid, block, 0, stream, A, lda, Wp, ldw, Cp, ldc, M, N, K, re,
                           nullptr, nullptr);
    }
  }
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

static int gemm_fp8_launch(const void* a, int64_t lda, const float* a_scale, const void* w, int64_t ldw,
                           const float* w_scale, void* c, int64_t ldc, int M, int N, int K, int epilogue,
                           const ResEpi& re, hipStream_t stream) {
  if (!a || !w || !c || !a_scale || !w_scale || M <= 0 || N <= 0 || K <= 0) return CP25_ERR_INVAL;
  if (N % kBN != 0 || K % 256 != 0) return CP25_ERR_DTYPE;  // 256-wide output tiles, an even number of 128-deep K-tiles
  if (lda < K || ldw < K || ldc < N || (lda % 16) || (ldw % 16) || (ldc % 8)) return CP25_ERR_INVAL;
  if (lda >= (1 << 23) || ldw >= (1 << 23)) return CP25_ERR_INVAL;
  if (((uintptr_t)a | (uintptr_t)w | (uintptr_t)c) & 15 || ((uintptr_t)a_scale | (uintptr_t)w_scale) & 3)
    return CP25_ERR_INVAL;
  if (epilogue != CP25_EPI_NONE && epilogue != CP25_EPI_RES) return CP25_ERR_INVAL;
  if (epilogue == CP25_EPI_RES &&
      (!re.x || !re.gate || re.B <= 0 || 16 % re.B || re.hw < 16 / re.B || re.tok0 < 0 || (re.x_st % 8) ||
       (re.x_sb % 8) || (re.g_sb % 8) || (re.g_st % 8) || (((uintptr_t)re.x | (uintptr_t)re.gate) & 15)))
    return CP25_ERR_INVAL;
  const int64_t nwg = (int64_t)((M + kBM - 1) / kBM) * (N / kBN);
  if (nwg > 0x7fffffff) return CP25_ERR_INVAL;
  static int n_cu[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return CP25_ERR_LAUNCH;
  if (!n_cu[dev] && hipDeviceGetAttribute(&n_cu[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return CP25_ERR_LAUNCH;
  const int cus = n_cu[dev] >= 8 ? n_cu[dev] & ~7 : n_cu[dev];
  const dim3 pgrid((unsigned)std::min<int64_t>(4 * nwg, cus)), block(kThreads);  // (tail row slices: gemm_launch)
  auto* A = (const unsigned short*)a;
  auto* Wp = (const unsigned short*)w;
  auto* Cp = (unsigned short*)c;
  if (epilogue == CP25_EPI_RES)
    hipLaunchKernelGGL((gemm_nt_8ph<CP25_EPI_RES, 1>), pgrid, block, 0, stream, A, lda, Wp, ldw, Cp, ldc, M, N, K, re,
                       a_scale, w_scale);
  else
    hipLaunchKernelGGL((gemm_nt_8ph<CP25_EPI_NONE, 1>), pgrid, block, 0, stream, A, lda, Wp, ldw, Cp, ldc, M, N, K, re,
                       a_scale, w_scale);
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

extern "C" int cp25_gemm_fp8(const void* a, int64_t lda, const float* a_scale, const void* w, int64_t ldw,
                             const float* w_scale, void* c, int64_t ldc, int M, int N, int K, hipStream_t stream) {
  const ResEpi re{};
  return gemm_fp8_launch(a, lda, a_scale, w, ldw, w_scale, c, ldc, M, N, K, CP25_EPI_NONE, re, stream);
}

extern "C" int cp25_gemm_fp8_res(const void* a, int64_t lda, const float* a_scale, const void* w, int64_t ldw,
                                 const float* w_scale, void* c, int64_t ldc, int M, int N, int K, const void* x,
                                 int64_t x_st, int64_t x_sb, const void* gate, int64_t g_sb, int64_t g_st, int B,
                                 int64_t tok0, int64_t hw, hipStream_t stream) {
  const ResEpi re{(const unsigned short*)x, x_st, x_sb, (const unsigned short*)gate, g_sb, g_st, B, tok0, hw};
  return gemm_fp8_launch(a, lda, a_scale, w, ldw, w_scale, c, ldc, M, N, K, CP25_EPI_RES, re, stream);
}

extern "C" int cp25_gemm_hnorm(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int M,
                               int N, int K, const void* norm_weight, float eps, float out_scale, hipStream_t stream) {
  ResEpi re{};
  re.nw = (const unsigned short*)norm_weight;
  re.n_eps = eps;
  re.n_scale = out_scale;
  return gemm_launch(a, lda, w, ldw, c, ldc, M, N, K, CP25_EPI_HNORM, re, stream);
}

extern "C" int cp25_gemm_qkv(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int M,
                             int N, int K, int k_col0, int k_cols, const void* k_norm_weight, const float* cos_tab,
                             const float* sin_tab, int B, float eps, hipStream_t stream) {
  ResEpi re{};
  re.nw = (const unsigned short*)k_norm_weight;
  re.n_eps = eps;
  re.n_scale = 1.f;
  re.rcos = cos_tab;
  re.rsin = sin_tab;
  re.B = B;
  re.n_lo = k_col0;
  re.n_hi = k_col0 + k_cols;
  return gemm_launch(a, lda, w, ldw, c, ldc, M, N, K, CP25_EPI_QKV, re, stream);
}

extern "C" int cp25_gemm_epi(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int M,
                             int N, int K, int epilogue, hipStream_t stream) {
  if (epilogue == CP25_EPI_RES || epilogue == CP25_EPI_HNORM || epilogue == CP25_EPI_QKV)
    return CP25_ERR_INVAL;  // their operands: _res / _hnorm / _qkv
  const ResEpi re{};
  return gemm_launch(a, lda, w, ldw, c, ldc, M, N, K, epilogue, re, stream);
}

extern "C" int cp25_gemm_res(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int M,
                             int N, int K, const void* x, int64_t x_st, int64_t x_sb, const void* gate, int64_t g_sb,
                             int64_t g_st, int B, int64_t tok0, int64_t hw, hipStream_t stream) {
  const ResEpi re{(const unsigned short*)x, x_st, x_sb, (const unsigned short*)gate, g_sb, g_st, B, tok0, hw};
  return gemm_launch(a, lda, w, ldw, c, ldc, M, N, K, CP25_EPI_RES, re, stream);
}
