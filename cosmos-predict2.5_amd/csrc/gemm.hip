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
//
// Design (MI355X, see DESIGN.md §3 "GEMM"): 256 x 256 output tile per 512-thread workgroup (one per
// CU), 8 waves as 2 (M) x 4 (N), each wave 128 x 64 with v_mfma_f32_16x16x32_bf16 (32 accumulators,
// the MFMA shape that holds the higher clock under load, MI355X_MICROARCH "DVFS" item 7); K in 64-deep
// tiles staged global -> LDS by LDS-DMA (global_load_lds_dwordx4, one 1-KiB piece = 8 rows x 128 B per
// wave instruction) into two buffers: tile k+1's DMA is in flight while tile k is multiplied. The LDS
// image is XOR-swizzled on the SOURCE side (16-B chunk c of row r lands at chunk c ^ ((r >> 1) & 7)),
// which makes every ds_read_b128 fragment read bank-conflict-free. Tiles are walked XCD-aware and
// grouped (8 row-tiles x all column tiles per group) so the workgroups resident on one XCD share
// their A and W tiles through that XCD's L2. Rows past M are clamped on load and masked on store.
// The epilogue stages each wave's bf16 tile through LDS and writes whole 16-B row chunks.
#include "cp25_common.h"

#pragma clang fp contract(off)

namespace {

constexpr int kBM = 256, kBN = 256, kBK = 64;
constexpr int kThreads = 512;
constexpr int kTileBytes = kBM * kBK * 2;       // 32 KiB per operand tile
constexpr int kStage = 2 * kTileBytes;          // A | W
constexpr int kLds = 2 * kStage;                // two stages: 128 KiB
constexpr int kGroupM = 8;

typedef __attribute__((address_space(3))) void* lds_void_ptr;

__device__ __forceinline__ float gelu_exact(float a) {
  return 0.5f * a * (1.f + erff(a * 0.70710678118654752440f));  // = cp25_gelu
}

template <int kEpi>
__global__ void __launch_bounds__(kThreads, 1)
gemm_nt_kernel(const unsigned short* __restrict__ A, int64_t lda, const unsigned short* __restrict__ W, int64_t ldw,
               unsigned short* __restrict__ C, int64_t ldc, int M, int N, int K) {
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
    if (row0 + r < M)
      *reinterpret_cast<u32x4*>(C + (int64_t)(row0 + r) * ldc + col0 + ch * 8) =
          *reinterpret_cast<const u32x4*>(st + r * 64 + ch * 8);
  }
}

}  // namespace

extern "C" int cp25_gemm_epi(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int M,
                             int N, int K, int epilogue, hipStream_t stream) {
  if (!a || !w || !c || M <= 0 || N <= 0 || K <= 0) return CP25_ERR_INVAL;
  if (N % kBN != 0 || K % kBK != 0) return CP25_ERR_DTYPE;  // the tiles this kernel is built for
  if (lda < K || ldw < K || ldc < N || (lda % 8) || (ldw % 8) || (ldc % 8)) return CP25_ERR_INVAL;
  if (((uintptr_t)a | (uintptr_t)w | (uintptr_t)c) & 15) return CP25_ERR_INVAL;
  const int64_t nwg = (int64_t)((M + kBM - 1) / kBM) * (N / kBN);
  if (nwg > 0x7fffffff) return CP25_ERR_INVAL;
  const unsigned short* A = (const unsigned short*)a;
  const unsigned short* Wp = (const unsigned short*)w;
  unsigned short* Cp = (unsigned short*)c;
  if (epilogue == CP25_EPI_NONE)
    hipLaunchKernelGGL(gemm_nt_kernel<CP25_EPI_NONE>, dim3((unsigned)nwg), dim3(kThreads), 0, stream, A, lda, Wp, ldw,
                       Cp, ldc, M, N, K);
  else if (epilogue == CP25_EPI_GELU)
    hipLaunchKernelGGL(gemm_nt_kernel<CP25_EPI_GELU>, dim3((unsigned)nwg), dim3(kThreads), 0, stream, A, lda, Wp, ldw,
                       Cp, ldc, M, N, K);
  else
    return CP25_ERR_INVAL;
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}
