// Pieces shared by the self/cross-attention kernels (attn_fwd.hip: attn_fwd_m16, attn_fwd_f8, the host launch;
// attn_w64.hip: attn_fwd_w64): the argument block, the tile geometry and the small device helpers.
#pragma once
#include "cp25_common.h"

#include <algorithm>
#include <type_traits>

namespace cp25attn {

constexpr int kD = 128;        // head dim
constexpr int kWaves = 8;      // waves per workgroup
constexpr int kQRows = 32;     // query rows per wave
constexpr int kQBlk = kWaves * kQRows;  // 256 query rows per workgroup
constexpr int kKBlk = 64;      // keys per tile
constexpr int kThreads = kWaves * 64;
// Softmax-shift ranges (log2 units). A term is 2^(s - shift) <= 2^kTop, so a row sum is <= Lk 2^96 and O = sum P v is
// <= Lk 2^96 max|v|: inside fp32 (2^128) while max|v| Lk < 2^32, e.g. |v| < 2.6e4 at config 4's Lk = 163 800 (the
// DiT's v is a bf16 projection of a normalised row, orders of magnitude smaller; checked at the top of the window
// over 163 840 keys with |v| ~ 400 by tests/test_attn_m16_gpu.py::test_m16_zero_shift_top_of_window_long_keys). The
// contract guard below poisons a row whose sum overflows. bf16 P has the fp32 exponent range.
constexpr float kTop = 96.f;        // zero / fixed shift: largest exponent a term may reach
constexpr float kMaxBound = 98.f;   // fixed shift: largest score bound b (smallest row-max term 2^(96 - 2 b) >= 2^-100)
constexpr float kPDrop = 60.f;      // fixed shift (round 6): rows shift by floor(min(b_row + 60, 126 - b_row)), so
                                    // P <= 2^-59 where b_row <= 33 and P <= 2^(2 b_row - 125) past it, the row's
                                    // largest term >= 2^-126. Small P runs the power-limited loop faster (P <= 2 vs
                                    // 2^17: -0.8 %; 2^-59 vs 2: -0.7 %, profiles/r6/shift_power/)
constexpr float kGateFixed = 110.f; // gated pair: a block whose data-tight bound is <= 110 runs the fixed shift, whose
                                    // rows then keep P <= 2^(2 * 110 - 125) = 2^95 (inside the zero-shift window's 2^96)
constexpr float kTopF8 = 60.f;      // fp8 Q K^T form: P = exp2(S) unshifted for bound products up to this
constexpr float kLazy = 24.f;       // online max: rescale only when a row max exceeds the shift by more (P <= 2^24)

typedef __attribute__((address_space(3))) const char* lds_char_ptr;

// cp25_common.h's hn_* pieces on element pairs (v_pk_* f32): per element the same IEEE operations, contraction off
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 hn2_sumsq8(const f32x2* x) {  // two sequential 8-term chains
#pragma clang fp contract(off)
  f32x2 ss = {0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 8; ++e) ss += x[e] * x[e];
  return ss;
}
__device__ __forceinline__ f32x2 hn2_norm(f32x2 x, f32x2 rstd, f32x2 w) {
#pragma clang fp contract(off)
  const f32x2 t = (x * rstd) * w;
  return __builtin_convertvector(__builtin_convertvector(t, bf16x2v), f32x2);  // rbf
}
__device__ __forceinline__ f32x2 hn2_rope(f32x2 v, f32x2 partner, float sgn, f32x2 c, f32x2 s) {
#pragma clang fp contract(off)
  const f32x2 sg = {sgn, sgn};
  return __builtin_elementwise_fma(v, c, (sg * partner) * s);
}

// compile-time loop: f(integral_constant<int, I>) for I = 0 .. N-1, in order
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

// The lane index computed afresh where it is used (opaque to CSE / loop-invariant hoisting): the persistent form
// recomputes its lane-dependent addresses per use instead of holding them in VGPRs across the tile loop, where a
// 256-VGPR kernel would spill them and reload them behind a vmcnt(0) that drains the tile loads in flight.
__device__ __forceinline__ int lane_fresh() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

__device__ __forceinline__ float wave_swap_sum(float x) {  // lanes l and l ^ 32
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float group4_sum(float x) {  // over the 4 lane groups of 16 (lanes c, c+16, c+32, c+48)
  x += __shfl_xor(x, 16);
  return x + __shfl_xor(x, 32);
}
__device__ __forceinline__ float group4_max(float x) {  // the same reduction by row swaps (no LDS crossbar)
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
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
  int ntk_v;        // fp8 P.V: key tiles per (b, h) of the v8t layout (ceil(Lk / 64))
  const float* v_amax;  // fp8 P.V: per-(b, h) max |v| (v8t holds v * 448 / amax)
  float s_init;     // fp8 forms: the Q K^T chains' initial C (-shift: P = exp2(S - shift) stays inside e5m2)
  float* o_part;    // nsplit > 1: [nsplit][B][H][Lq][128] fp32 partial O (normalised per split)
  float* lse_part;  // nsplit > 1: [nsplit][B][H][Lq] fp32 log2-sum-exp2 of the scaled scores
  float scale_log2; // softmax scale * log2(e) (1 for a pre-scaled q)
  float kbound;     // > 0: upper bound of |k| over all keys (fixed shift where it allows); 0: online max only
  const float* kslots;  // gated pair: max |k| over all keys = the max of n_kslots floats kslots[32 i] (device memory)
  int n_kslots;
  // in-kernel q normalisation (cp25_attn_fwd_prescaled_qnorm, per-block forms): q holds the raw projection; each
  // workgroup applies the per-head RMSNorm (weight qn_w[128], eps), the rotate-half RoPE of token qn_row0 + row
  // (qn_cos / qn_sin [tokens][64] fp32; nullptr: none) and the factor qn_scale to its Q fragments as they load.
  const unsigned short* qn_w;
  const float* qn_cos;
  const float* qn_sin;
  float qn_eps, qn_scale;
  int qn_row0;
#ifdef CP25_ATTN_PROBE
  // lab build only (tools/attn_probe.py; the product build has no stamp): [probe_wg][8 waves][32 tiles][4] s_memtime
  // stamps of workgroups blockIdx.x < probe_wg, tiles probe_t0 .. probe_t0 + 31
  unsigned long long* probe;
  int probe_t0, probe_wg;
#endif
};

// LDS image of a 64-key K or V tile: rows of 288 B (256 + 32; conflict-free ds_read_b128 K fragments and transposed
// ds_read_b64_tr_b16 V^T reads, attn_fwd_m16's header), two buffers each
constexpr int kKStride16 = 288;
constexpr int kVStride16 = 288;
constexpr int kKBuf16 = kKBlk * kKStride16;        // 18432
constexpr int kVBuf16 = kKBlk * kVStride16;        // 18432
constexpr int kLds16 = 2 * kKBuf16 + 2 * kVBuf16;  // 73728

// attn_fwd_w64 (attn_w64.hip): the kernel for a softmax mode (0 fixed, 1 zero shift, 2 online max) and symbol (tail
// segments separate in profiles)
typedef void (*AttnKernel)(AttnArgs);
AttnKernel w64_kernel(int mode, bool tail);
constexpr int kW64Threads = 256;  // 4 waves, one per SIMD

}  // namespace cp25attn
