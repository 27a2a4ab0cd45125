// fp8 (OCP E4M3, gfx950's native fp8 format) activation quantisation for the DiT's fp8 linear layers
// (BASELINE config 5, "fp8 MFMA"). The GEMMs themselves run on hipBLASLt's fp8 MFMA kernels through
// torch._scaled_mm with a per-row activation scale and a per-output-channel weight scale; these
// kernels produce the row-scaled activation operand.
//
//   cp25_quant_fp8_rows : x bf16 [M, K] -> q fp8 [M, K], s fp32 [M], x[m, k] ~= q[m, k] * s[m]
//   cp25_gelu_quant_fp8 : the same over GELU(x) (minimal_v4_dit.py:249-254; a 7.1.26-erfc GELU within
//                         ~1 bf16 ulp of the exact one, rounded to bf16 first), so the MLP's hidden
//                         activation is read once and never written back in bf16
//
// The reference has no fp8 inference path: these are the build's own (config-5) precision option,
// parity stated against the bf16 path in DESIGN.md §4, not a restatement of a reference kernel.
// One to four waves per row; the row stays in registers between the amax reduction and the conversion, so
// the kernels are one HBM read of x (2 B/element) and one write of q (1 B/element).
#include "cp25_common.h"

#pragma clang fp contract(off)

namespace {

constexpr float kFp8Max = 448.f;  // largest finite OCP E4M3 value

// GELU for the fp8 operand: x * Phi(x) with Phi from the Abramowitz-Stegun 7.1.26 erfc form
// erfc(z) = t (a1 + t (a2 + ...)) exp(-z^2), t = 1 / (1 + p z) (|error| <= 1.5e-7): ~14 VALU ops
// (two of them transcendental) instead of libm erff's ~39; Phi(x < 0) = erfc / 2 is taken directly,
// so there is no 1 + erf cancellation for negative inputs. Far below the fp8 rounding (2^-4) and
// within ~1 bf16 ulp of the exact-erf GELU (the bf16 path keeps libm erff, cp25_gelu).
__device__ __forceinline__ float gelu_fp8_operand(float a) {
  const float z = fabsf(a) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  const float poly =
      t * fmaf(fmaf(fmaf(fmaf(1.061405429f, t, -1.453152027f), t, 1.421413741f), t, -0.284496736f), t, 0.254829592f);
  const float ec = poly * __builtin_amdgcn_exp2f(-(z * z) * 1.44269504088896340736f);  // erfc(z)
  return a * (a >= 0.f ? 1.f - 0.5f * ec : 0.5f * ec);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
  return v;
}

// WPR waves per row (NW / WPR rows per NW-wave block), NC chunks of 8 values per lane:
// K = NC * WPR * 512; chunk c of wave w covers elements [(c * WPR + w) * 512 + lane * 8, +8).
// The longest rows (K = 20480, 14B's MLP hidden) spread over 8 waves so each lane keeps few values.
template <int WPR, int NC, bool GELU, int NW = 4>
__global__ void __launch_bounds__(NW * 64) quant_fp8_rows_kernel(const unsigned short* __restrict__ x,
                                                                 unsigned char* __restrict__ q,
                                                                 float* __restrict__ s, int64_t n_rows) {
  constexpr int K = NC * WPR * 512;
  __shared__ float red[NW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave % WPR;  // wave within its row
  const int64_t row = (int64_t)blockIdx.x * (NW / WPR) + wave / WPR;
  const bool live = row < n_rows;  // no early exit: the block meets at a barrier below
  const int64_t base = row * K + (int64_t)wr * 512 + lane * 8;
  // the row slice lives in registers as packed bf16 pairs (4 VGPRs per chunk) between the two passes
  u32x4 v[NC];
  float amax = 0.f;
  if (live) {
#pragma unroll
    for (int c = 0; c < NC; ++c) v[c] = *reinterpret_cast<const u32x4*>(x + base + c * WPR * 512);
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        float lo = __uint_as_float(v[c][w] << 16), hi = __uint_as_float(v[c][w] & 0xffff0000u);
        if constexpr (GELU) {
          lo = rbf(gelu_fp8_operand(lo));
          hi = rbf(gelu_fp8_operand(hi));
          v[c][w] = (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xffff0000u);
        }
        amax = fmaxf(amax, fmaxf(fabsf(lo), fabsf(hi)));
      }
  }
  amax = wave_max(amax);
  if constexpr (WPR > 1) {
    if (lane == 0) red[wave] = amax;
    __syncthreads();
    const int w0 = wave - wr;
#pragma unroll
    for (int j = 0; j < WPR; ++j) amax = fmaxf(amax, red[w0 + j]);
  }
  if (!live) return;
  const float inv = amax > 0.f ? kFp8Max / amax : 0.f;
  if (lane == 0 && wr == 0) s[row] = amax / kFp8Max;
  unsigned char* qr = q + base;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    u32x2 o;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float f[4];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const unsigned w = v[c][2 * h + e];
        f[2 * e] = fminf(fmaxf(__uint_as_float(w << 16) * inv, -kFp8Max), kFp8Max);
        f[2 * e + 1] = fminf(fmaxf(__uint_as_float(w & 0xffff0000u) * inv, -kFp8Max), kFp8Max);
      }
      int w = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
      w = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], w, true);
      o[h] = (unsigned)w;
    }
    *reinterpret_cast<u32x2*>(qr + c * WPR * 512) = o;
  }
}

template <int WPR, int NC, bool GELU, int NW = 4>
void launch_rows(const unsigned short* x, unsigned char* q, float* s, int64_t n_rows, hipStream_t stream) {
  hipLaunchKernelGGL((quant_fp8_rows_kernel<WPR, NC, GELU, NW>), dim3((unsigned)cdiv(n_rows, NW / WPR)),
                     dim3(NW * 64), 0, stream, x, q, s, n_rows);
}

template <bool GELU>
int launch_quant(const void* x, void* q, float* s, int64_t n_rows, int64_t k, hipStream_t stream) {
  if (!x || !q || !s || n_rows <= 0) return CP25_ERR_INVAL;
  const auto* xp = (const unsigned short*)x;
  auto* qp = (unsigned char*)q;
  switch (k) {
    case 512: launch_rows<1, 1, GELU>(xp, qp, s, n_rows, stream); break;
    case 1024: launch_rows<1, 2, GELU>(xp, qp, s, n_rows, stream); break;
    case 1536: launch_rows<1, 3, GELU>(xp, qp, s, n_rows, stream); break;
    case 2048: launch_rows<1, 4, GELU>(xp, qp, s, n_rows, stream); break;
    case 3072: launch_rows<2, 3, GELU>(xp, qp, s, n_rows, stream); break;
    case 4096: launch_rows<2, 4, GELU>(xp, qp, s, n_rows, stream); break;
    case 5120: launch_rows<2, 5, GELU>(xp, qp, s, n_rows, stream); break;
    case 6144: launch_rows<4, 3, GELU>(xp, qp, s, n_rows, stream); break;
    // 4 waves x 4 chunks per lane: 1.46 ms at [218240, 8192] vs 1.68 (16 x 1) and 1.52 (8 x 2)
    case 8192: launch_rows<4, 4, GELU>(xp, qp, s, n_rows, stream); break;
    case 20480: launch_rows<8, 5, GELU, 8>(xp, qp, s, n_rows, stream); break;
    default: return CP25_ERR_INVAL;
  }
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

// dst[r, c] = e4m3(bf16 src[r, c] * scale), saturated to +-448, round to nearest even: the fixed power-of-two
// scaled fp8 copy of q and k for cp25_attn_fwd_prescaled_fp8qk. One thread per 16 elements (two 16-B loads,
// one 16-B store); width % 16 == 0. HBM-bound.
__global__ void __launch_bounds__(256) cast_fp8_kernel(const unsigned short* __restrict__ src, int64_t src_stride,
                                                       unsigned char* __restrict__ dst, int64_t dst_stride,
                                                       int64_t n_rows, int cpr, float scale) {
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= n_rows * cpr) return;
  const int64_t r = gid / cpr;
  const int c = (int)(gid % cpr) * 16;
  const u32x4 a = *reinterpret_cast<const u32x4*>(src + r * src_stride + c);
  const u32x4 b = *reinterpret_cast<const u32x4*>(src + r * src_stride + c + 8);
  u32x4 o;
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const unsigned w0 = h < 2 ? a[2 * h] : b[2 * h - 4], w1 = h < 2 ? a[2 * h + 1] : b[2 * h - 3];
    float f[4] = {__uint_as_float(w0 << 16), __uint_as_float(w0 & 0xffff0000u), __uint_as_float(w1 << 16),
                  __uint_as_float(w1 & 0xffff0000u)};
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = fminf(fmaxf(f[e] * scale, -kFp8Max), kFp8Max);
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], w, true);
    o[h] = (unsigned)w;
  }
  *reinterpret_cast<u32x4*>(dst + r * dst_stride + c) = o;
}

// ---- V for the fp8 P.V of cp25_attn_fwd_prescaled_fp8: per-(b, h) amax, then an e4m3 copy laid out as the MFMA's
// A operand wants it. v_mfma_f32_32x32x64_f8f6f4 with A = V^T (32 d rows x 64 keys) and B = P^T (64 keys x 32
// queries): lane half hl, byte j of both operands must name the same key. The P^T operand is the S^T accumulator
// as it lies in the lane (S[kt][r]: key 32 kt + (r & 3) + 8 (r >> 2) + 4 hl, byte j = 16 kt + r), so a V^T row d
// of a 64-key tile is stored as 64 bytes p = 32 hl + j holding V[key(j, hl)][d] / scale: v8t[b][h][tile][d][p].
// One lane then reads its 32-byte fragment contiguously (two ds_read_b128). Keys past L are zero.
__device__ __forceinline__ int vt_key(int p) {
  const int hl = p >> 5, j = p & 31;
  return 32 * (j >> 4) + (j & 3) + 8 * ((j >> 2) & 3) + 4 * hl;
}

// amax[b * H + h] = max |v| over the L rows of head (b, h) (float bits, atomicMax on non-negative floats as uints).
// grid (B * H, nchunk), 256 threads: thread t reads 16-B chunk t % 16 of rows t / 16 + 16 i.
__global__ void __launch_bounds__(256) v_amax_kernel(const unsigned short* __restrict__ v, int64_t sb, int64_t sl,
                                                     int64_t sh, int H, int L, int rows_per_chunk,
                                                     unsigned* __restrict__ amax) {
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const unsigned short* vp = v + b * sb + h * sh;
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(L, r0 + rows_per_chunk);
  float m = 0.f;
  for (int r = r0 + (threadIdx.x >> 4); r < r1; r += 16) {
    const u32x4 w = *reinterpret_cast<const u32x4*>(vp + (int64_t)r * sl + 8 * (threadIdx.x & 15));
#pragma unroll
    for (int e = 0; e < 4; ++e)
      m = fmaxf(m, fmaxf(fabsf(__uint_as_float(w[e] << 16)), fabsf(__uint_as_float(w[e] & 0xffff0000u))));
  }
  m = wave_max(m);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(amax + bh, __float_as_uint(m));
  }
}

// v8t tile (b, h, tile): 64 keys x 128 d bf16 through LDS, out as [128 d][64 p] e4m3 of v / scale,
// scale = max(amax, 2^-100) / 448 (also what the attention multiplies O by). grid (B * H, ntile), 256 threads.
__global__ void __launch_bounds__(256) v_cast_t_kernel(const unsigned short* __restrict__ v, int64_t sb, int64_t sl,
                                                       int64_t sh, int H, int L, int ntile,
                                                       const unsigned* __restrict__ amax,
                                                       unsigned char* __restrict__ v8t) {
  constexpr int RS = 128 + 8;  // LDS row stride (bf16 elements)
  __shared__ unsigned short t[64 * RS];
  const int bh = blockIdx.x, b = bh / H, h = bh % H, tile = blockIdx.y;
  const unsigned short* vp = v + b * sb + h * sh;
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // 1024 chunks of 8 bf16: key c / 16, d 8 (c % 16)
    const int c = threadIdx.x + 256 * i, key = c >> 4, d0 = 8 * (c & 15), row = 64 * tile + key;
    u32x4 w = {0u, 0u, 0u, 0u};
    if (row < L) w = *reinterpret_cast<const u32x4*>(vp + (int64_t)row * sl + d0);
    *reinterpret_cast<u32x4*>(t + key * RS + d0) = w;
  }
  __syncthreads();
  const float inv = 448.f / fmaxf(__uint_as_float(amax[bh]), 0x1p-100f);
  unsigned char* out = v8t + ((int64_t)bh * ntile + tile) * 8192;
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // 512 output chunks of 16 B: d = c / 4, p0 = 16 (c % 4)
    const int c = threadIdx.x + 256 * i, d = c >> 2, p0 = 16 * (c & 3);
    u32x4 o;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      float f[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const unsigned short x = t[vt_key(p0 + 4 * w + e) * RS + d];
        f[e] = fminf(fmaxf(__uint_as_float((unsigned)x << 16) * inv, -kFp8Max), kFp8Max);
      }
      int q = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
      q = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], q, true);
      o[w] = (unsigned)q;
    }
    *reinterpret_cast<u32x4*>(out + d * 64 + p0) = o;
  }
}

}  // namespace

extern "C" int64_t cp25_v_fp8t_bytes(int B, int H, int L) {
  if (B <= 0 || H <= 0 || L <= 0) return CP25_ERR_INVAL;
  return (int64_t)B * H * cdiv(L, 64) * 8192;
}

extern "C" int cp25_cast_v_fp8t(const void* v, const int64_t* v_strides, int B, int H, int L, int D, void* v8t,
                                float* v_amax, hipStream_t stream) {
  if (!v || !v_strides || !v8t || !v_amax || B <= 0 || H <= 0 || L <= 0) return CP25_ERR_INVAL;
  if (D != 128) return CP25_ERR_DTYPE;
  for (int j = 0; j < 3; ++j)
    if (v_strides[j] % 8) return CP25_ERR_INVAL;
  if ((((uintptr_t)v) | ((uintptr_t)v8t)) & 15) return CP25_ERR_INVAL;
  const int ntile = (int)cdiv(L, 64);
  unsigned* amax = reinterpret_cast<unsigned*>(v_amax);
  if (hipMemsetAsync(amax, 0, sizeof(unsigned) * B * H, stream) != hipSuccess) return CP25_ERR_LAUNCH;
  const int rows_per_chunk = 1024, nchunk = (int)cdiv(L, rows_per_chunk);
  hipLaunchKernelGGL(v_amax_kernel, dim3(B * H, nchunk), dim3(256), 0, stream, (const unsigned short*)v, v_strides[0],
                     v_strides[1], v_strides[2], H, L, rows_per_chunk, amax);
  CP25_LAUNCH_CHECK();
  hipLaunchKernelGGL(v_cast_t_kernel, dim3(B * H, ntile), dim3(256), 0, stream, (const unsigned short*)v, v_strides[0],
                     v_strides[1], v_strides[2], H, L, ntile, (const unsigned*)amax, (unsigned char*)v8t);
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

extern "C" int cp25_cast_fp8_e4m3(const void* src, int64_t src_stride, void* dst, int64_t dst_stride, int64_t n_rows,
                                  int64_t width, float scale, hipStream_t stream) {
  if (!src || !dst || n_rows <= 0 || width <= 0 || width % 16 || src_stride < width || dst_stride < width ||
      (src_stride % 8) || (dst_stride % 16) || (((uintptr_t)src | (uintptr_t)dst) & 15) || !(scale > 0.f))
    return CP25_ERR_INVAL;
  const int cpr = (int)(width / 16);
  const int64_t n = n_rows * cpr;
  hipLaunchKernelGGL(cast_fp8_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, (const unsigned short*)src,
                     src_stride, (unsigned char*)dst, dst_stride, n_rows, cpr, scale);
  CP25_LAUNCH_CHECK();
  return CP25_OK;
}

extern "C" int cp25_quant_fp8_rows(const void* x, void* q, float* scale, int64_t n_rows, int64_t k,
                                   hipStream_t stream) {
  return launch_quant<false>(x, q, scale, n_rows, k, stream);
}

extern "C" int cp25_gelu_quant_fp8(const void* x, void* q, float* scale, int64_t n_rows, int64_t k,
                                   hipStream_t stream) {
  return launch_quant<true>(x, q, scale, n_rows, k, stream);
}
