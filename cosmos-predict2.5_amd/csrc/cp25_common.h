// Shared device/host helpers for the cosmos-predict2.5 MI355X kernels (gfx950 only).
//
// Conventions used by every entry point in include/cp25.h:
//   * tensors are device pointers + element strides; the caller (PyTorch's caching
//     allocator on the Python side) owns all memory, kernels never allocate;
//   * every call is stream-ordered on the hipStream_t passed in, never synchronises,
//     and is safe to capture into a hipGraph;
//   * return 0 on success, a negative errno-style code on bad arguments (checked on the
//     host before any launch), or CP25_ERR_LAUNCH if the launch itself failed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "cp25.h"

#define CP25_OK 0
#define CP25_ERR_INVAL (-22)   /* bad shape / stride / size */
#define CP25_ERR_DTYPE (-95)   /* unsupported dtype / head dim */
#define CP25_ERR_LAUNCH (-5)   /* hipLaunch failure */

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// bf16 <-> f32 with round-to-nearest-even (matches torch's .to(bfloat16)).
__device__ __forceinline__ float bf2f(unsigned short b) { return __uint_as_float(((unsigned)b) << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
  // plain conversion: hipcc lowers it to v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950
  __bf16 h = static_cast<__bf16>(f);
  return __builtin_bit_cast(unsigned short, h);
}
// round an f32 to the nearest bf16 value and return it as f32 (emulates a bf16 tensor op)
__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }

__host__ __device__ __forceinline__ int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// XCD-aware bijective remap of a 1-D grid: blocks b and b+8 share an XCD, so give each
// group of 8 a contiguous range of logical tiles (cdna_hip_programming.md §5 T1).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

#define CP25_LAUNCH_CHECK()                                     \
  do {                                                          \
    if (hipGetLastError() != hipSuccess) return CP25_ERR_LAUNCH; \
  } while (0)
