// fp32 linear layers of the DiT's fp32-autocast pieces (gfx950):
//   C[b][M, N] = act(A[b][M, K] W[b][N, K]^T + R[b][M, N])        (fp32 in / out, act: none or SiLU)
// with an optional addend R read through its own strides (row stride 0: a bias vector; batch stride 0: one matrix
// for every batch entry), added to the fp32 accumulator as the reference's separate fp32 `+` would.
// replacing the reference's fp32 F.linear calls (use_wan_fp32_strategy, networks/minimal_v4_dit.py):
//   * the t-embedding MLP, TimestepEmbedding linear_1 + SiLU and linear_2 (:727-788);
//   * the blocks' AdaLN-LoRA modulation, Sequential(SiLU, Linear(D, A), Linear(A, 3D)) per sub-layer (:1136-1154),
//     the first Linear of all 28 x 3 sub-layers as one GEMM and the second as one batched GEMM (batch = sub-layer);
//   * the final layer's AdaLN (:974-991) and its Linear(D, p p C) on every token (:993-995).
// v_mfma_f32_16x16x4_f32: f32 operands, products and sums (the fp32 FMA chain of each k slot; no reduced-precision
// input), so the only difference from any other fp32 GEMM is the summation order.
//
// Tile: 128 rows x 64 columns per 256-thread workgroup (64 rows when M <= 64: the 62-row conditioning GEMMs), K in
// chunks of 32. Wave w owns 32 (16) rows, two (one) 16-row blocks, and all 64 columns (four 16-column blocks). The W chunk [64][32] goes
// through the LDS (rows of 36 floats: the float4 B-fragment reads of 16 lanes land on 16 disjoint 4-bank groups); A is
// read straight from global memory as float4 fragments (each A element is used by this workgroup only). K slot g of
// the MFMA holds k = 16 ks + 4 g + s at step s for both operands, so a lane reads 4 consecutive k of its row.
#include "cp25_common.h"

namespace {

constexpr int kTM = 128, kTN = 64, kTK = 32;
constexpr int kWS = kTK + 4;  // LDS row stride (floats)

typedef float f32x4v __attribute__((ext_vector_type(4)));

template <int kAct, bool kAdd, bool kSplit, int kRB>
__global__ void __launch_bounds__(256) gemm_f32_kernel(const float* __restrict__ A, int64_t lda, int64_t sa,
                                                       const float* __restrict__ W, int64_t ldw, int64_t sw,
                                                       const float* __restrict__ R, int64_t ldr, int64_t sr,
                                                       float* __restrict__ C, int64_t ldc, int64_t sc, int M, int N,
                                                       int K, int splits) {
  __shared__ __attribute__((aligned(16))) float wt[2][kTN * kWS];
  // split-K: blockIdx.z = batch entry * splits + slice; the slice's partial sums go to the workspace C[slice][b]
  const int b = kSplit ? blockIdx.z / splits : blockIdx.z;
  const int slice = kSplit ? blockIdx.z % splits : 0;
  const int nk = K / kTK;
  const int c0 = kSplit ? (int)((int64_t)slice * nk / splits) : 0;
  const int c1 = kSplit ? (int)((int64_t)(slice + 1) * nk / splits) : nk;
  A += b * sa;
  W += b * sw;
  if constexpr (kSplit) {
    C += ((int64_t)slice * (gridDim.z / splits) + b) * sc;
  } else {
    C += b * sc;
  }
  if constexpr (kAdd) R += b * sr;
  const int m0 = blockIdx.x * 64 * kRB, n0 = blockIdx.y * kTN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, g = lane >> 4;
  // W chunk staging: thread t moves 8 floats, column t / 4, k (t % 4) 8 .. (columns past N clamped, not stored)
  const int wc = tid >> 2, wk = (tid & 3) * 8;
  const float* wsrc = W + (int64_t)min(n0 + wc, N - 1) * ldw + wk;
  // A fragments: rows of this wave's kRB row blocks (clamped: rows past M are computed and not stored)
  const float* asrc[kRB];
#pragma unroll
  for (int rb = 0; rb < kRB; ++rb)
    asrc[rb] = A + (int64_t)min(m0 + 16 * kRB * wave + 16 * rb + c16, M - 1) * lda + 4 * g;

  f32x4v acc[kRB][4];
#pragma unroll
  for (int rb = 0; rb < kRB; ++rb)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[rb][cb] = f32x4v{0.f, 0.f, 0.f, 0.f};

  // one chunk ahead in registers, two LDS buffers: chunk c is stored to wt[c & 1] while the loads of c + 1 are in
  // flight; one barrier per chunk (the buffer written at c was last read at c - 2, before the barrier of c - 1)
  f32x4v w0, w1, af[2][kRB];
  auto load = [&](int c) {
    const int kc = c * kTK;
    w0 = *reinterpret_cast<const f32x4v*>(wsrc + kc);
    w1 = *reinterpret_cast<const f32x4v*>(wsrc + kc + 4);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int rb = 0; rb < kRB; ++rb) af[ks][rb] = *reinterpret_cast<const f32x4v*>(asrc[rb] + kc + 16 * ks);
  };
  load(c0);
  for (int c = c0; c < c1; ++c) {
    float* buf = wt[c & 1];
    *reinterpret_cast<f32x4v*>(buf + wc * kWS + wk) = w0;
    *reinterpret_cast<f32x4v*>(buf + wc * kWS + wk + 4) = w1;
    f32x4v a_cur[2][kRB];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int rb = 0; rb < kRB; ++rb) a_cur[ks][rb] = af[ks][rb];
    __syncthreads();
    if (c + 1 < c1) load(c + 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f32x4v bf[4];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
        bf[cb] = *reinterpret_cast<const f32x4v*>(buf + (16 * cb + c16) * kWS + 16 * ks + 4 * g);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int rb = 0; rb < kRB; ++rb)
#pragma unroll
          for (int cb = 0; cb < 4; ++cb)
            acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_cur[ks][rb][s], bf[cb][s], acc[rb][cb], 0, 0, 0);
    }
  }
  // lane holds D[4 g + i][c16] of each block: row m0 + 16 kRB wave + 16 rb + 4 g + i, column n0 + 16 cb + c16
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int col = n0 + 16 * cb + c16;
    if (col >= N) continue;
#pragma unroll
    for (int rb = 0; rb < kRB; ++rb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + 16 * kRB * wave + 16 * rb + 4 * g + i;
        if (row >= M) continue;
        float v = acc[rb][cb][i];
        if constexpr (!kSplit) {
          if constexpr (kAdd) v += R[(int64_t)row * ldr + col];
          if constexpr (kAct == 1) v = v / (1.f + expf(-v));  // SiLU, as torch's fp32 F.silu: x * sigmoid(x)
        }
        C[(int64_t)row * ldc + col] = v;
      }
  }
}

// split-K second pass: C[b][m][n] = act(sum over slices in slice order of P[s][b][m][n] + R), P dense [s][b][M][N]
template <int kAct, bool kAdd>
__global__ void __launch_bounds__(256) gemm_f32_reduce(const float* __restrict__ P, int splits, const float* __restrict__ R,
                                                       int64_t ldr, int64_t sr, float* __restrict__ C, int64_t ldc,
                                                       int64_t sc, int M, int N, int batch) {
  const int64_t per = (int64_t)M * N, total = per * batch;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int b = (int)(i / per);
    const int64_t mn = i - b * per;
    const int row = (int)(mn / N), col = (int)(mn - (int64_t)row * N);
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += P[s * total + i];
    if constexpr (kAdd) v += R[b * sr + (int64_t)row * ldr + col];
    if constexpr (kAct == 1) v = v / (1.f + expf(-v));
    C[b * sc + (int64_t)row * ldc + col] = v;
  }
}

// Slices of K for a launch of mt x nt x batch tiles: enough workgroups to cover the CUs (one tile of a 62-row
// conditioning GEMM is K / 32 dependent chunks, latency-bound) without exceeding one resident round, at least two
// chunks per slice, at most 16 slices.
int rows_per_tile(int M) { return M <= 64 ? 64 : kTM; }

int splits_for(int M, int N, int K, int batch) {
  const int64_t wgs = cdiv(M, rows_per_tile(M)) * cdiv(N, kTN) * (int64_t)batch;
  const int nk = K / kTK;
  if (wgs >= 512 || nk < 4) return 1;
  int s = (int)(1024 / wgs);  // one round of resident workgroups (4 per CU at this register count): no tail round
  s = min(s, min(16, nk / 2));
  if ((int64_t)s * batch > 65535) s = 65535 / batch;
  return max(s, 1);
}

}  // namespace

extern "C" int64_t cp25_gemm_f32_workspace_floats(int M, int N, int K, int batch) {
  if (M <= 0 || N <= 0 || K <= 0 || batch <= 0 || K % kTK) return 0;
  const int s = splits_for(M, N, K, batch);
  return s > 1 ? (int64_t)s * batch * M * N : 0;
}

extern "C" int cp25_gemm_f32(const float* a, int64_t lda, int64_t a_batch_stride, const float* w, int64_t ldw,
                             int64_t w_batch_stride, const float* r, int64_t ldr, int64_t r_batch_stride, float* c,
                             int64_t ldc, int64_t c_batch_stride, int M, int N, int K, int batch, int act,
                             float* workspace, int64_t workspace_floats, hipStream_t stream) {
  if (!a || !w || !c || M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535) return CP25_ERR_INVAL;
  if (K % kTK) return CP25_ERR_DTYPE;  // the K chunk this kernel is built for
  if (act != 0 && act != 1) return CP25_ERR_INVAL;
  if (lda < K || ldw < K || ldc < N || ldr < 0 || (lda % 4) || (ldw % 4) || (a_batch_stride % 4) ||
      (w_batch_stride % 4))
    return CP25_ERR_INVAL;
  if (((uintptr_t)a | (uintptr_t)w) & 15) return CP25_ERR_INVAL;  // float4 operand reads
  if (((uintptr_t)c | (uintptr_t)r | (uintptr_t)workspace) & 3) return CP25_ERR_INVAL;
  const int rb = rows_per_tile(M) / 64;
  const int64_t mt = cdiv(M, 64 * rb);
  if (mt > 0x7fffffff) return CP25_ERR_INVAL;
  int splits = splits_for(M, N, K, batch);
  const int64_t need = (int64_t)splits * batch * M * N;
  if (splits > 1 && (!workspace || workspace_floats < need)) splits = 1;  // no workspace: one slice (same result
                                                                         // up to summation order)
  const dim3 block(256);
  if (splits == 1) {
    const dim3 grid((unsigned)mt, (unsigned)cdiv(N, kTN), (unsigned)batch);
#define CP25_F32_LAUNCH(ACT, ADD)                                                                                    \
  if (rb == 1)                                                                                                       \
    hipLaunchKernelGGL((gemm_f32_kernel<ACT, ADD, false, 1>), grid, block, 0, stream, a, lda, a_batch_stride, w, ldw, \
                       w_batch_stride, r, ldr, r_batch_stride, c, ldc, c_batch_stride, M, N, K, 1);                   \
  else                                                                                                               \
    hipLaunchKernelGGL((gemm_f32_kernel<ACT, ADD, false, 2>), grid, block, 0, stream, a, lda, a_batch_stride, w, ldw, \
                       w_batch_stride, r, ldr, r_batch_stride, c, ldc, c_batch_stride, M, N, K, 1)
    if (r) {
      if (act == 1) {
        CP25_F32_LAUNCH(1, true);
      } else {
        CP25_F32_LAUNCH(0, true);
      }
    } else {
      if (act == 1) {
        CP25_F32_LAUNCH(1, false);
      } else {
        CP25_F32_LAUNCH(0, false);
      }
    }
#undef CP25_F32_LAUNCH
  } else {
    const dim3 grid((unsigned)mt, (unsigned)cdiv(N, kTN), (unsigned)(batch * splits));
    if (rb == 1)
      hipLaunchKernelGGL((gemm_f32_kernel<0, false, true, 1>), grid, block, 0, stream, a, lda, a_batch_stride, w, ldw,
                         w_batch_stride, (const float*)nullptr, 0, 0, workspace, (int64_t)N, (int64_t)M * N, M, N, K,
                         splits);
    else
      hipLaunchKernelGGL((gemm_f32_kernel<0, false, true, 2>), grid, block, 0, stream, a, lda, a_batch_stride, w, ldw,
                         w_batch_stride, (const float*)nullptr, 0, 0, workspace, (int64_t)N, (int64_t)M * N, M, N, K,
                         splits);
    CP25_LAUNCH_CHECK();
    const int64_t total = (int64_t)batch * M * N;
    const int64_t rblocks = cdiv(total, 256);
    const unsigned rg = (unsigned)(rblocks < 4096 ? rblocks : 4096);
#define CP25_F32_REDUCE(ACT, ADD)                                                                                    \
  hipLaunchKernelGGL((gemm_f32_reduce<ACT, ADD>), dim3(rg), block, 0, stream, workspace, splits, r, ldr,              \
                     r_batch_stride, c, ldc, c_batch_stride, M, N, batch)
    if (r) {
      if (act == 1) {
        CP25_F32_REDUCE(1, true);
      } else {
        CP25_F32_REDUCE(0, true);
      }
    } else {
      if (act == 1) {
        CP25_F32_REDUCE(1, false);
      } else {
        CP25_F32_REDUCE(0, false);
      }
    }
#undef CP25_F32_REDUCE
  }
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}
