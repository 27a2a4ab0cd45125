// Lab: does MFMA throughput under sustained load depend on operand bit activity between consecutive MFMAs?
// 256 CUs x 8 waves run back-to-back v_mfma_f32_32x32x16_bf16 on register operands with random bf16 data.
//   pattern 0: A and B change every MFMA (8 distinct each)
//   pattern 1: A changes every MFMA, B every 8
//   pattern 2: A every 8, B every MFMA
//   pattern 3: A and B never change
//   pattern 4: pattern 0 on zero data
// Prints TFLOP/s per pattern (hipEvent timing). Build: hipcc --offload-arch=gfx950 -O3 -o mfma_power mfma_power.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int P>
__global__ void __launch_bounds__(512, 2) mfma_loop(const bf16x8* __restrict__ src, float* __restrict__ out, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = src[(i * 64 + lane) % 1024];
    b[i] = src[((i + 8) * 64 + lane) % 1024];
  }
  f32x16 acc[4] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 64; ++j) {
      const int ia = (P == 0 || P == 1 || P == 4) ? (j & 7) : (P == 2 ? (j >> 3) & 7 : 0);
      const int ib = (P == 0 || P == 2 || P == 4) ? (j & 7) : (P == 1 ? (j >> 3) & 7 : 0);
      acc[j & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ia], b[ib], acc[j & 3], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// pattern 5 / 6: the same FLOPs and the same 4096 outputs per wave as pattern 0 / 4 on v_mfma_f32_16x16x32_bf16
// (16 accumulators of 16 x 16, twice the MFMAs at half the FLOP each): the shape lever of MI355X_MICROARCH
// "DVFS give-back" item 7
template <int P>
__global__ void __launch_bounds__(512, 2) mfma_loop16(const bf16x8* __restrict__ src, float* __restrict__ out, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = src[(i * 64 + lane) % 1024];
    b[i] = src[((i + 8) * 64 + lane) % 1024];
  }
  f32x4 acc[16] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 128; ++j)
      acc[j & 15] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j & 7], b[(j >> 1) & 7], acc[j & 15], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 16; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) s += acc[c][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// pattern 7 / 8: block-scaled fp8 (e4m3) MFMAs on random bytes, same 4096 outputs per wave:
// 7 = v_mfma_scale_f32_32x32x64_f8f6f4 (4 accumulators of 32 x 32), 8 = v_mfma_scale_f32_16x16x128_f8f6f4 (16 of 16 x 16)
typedef int i32x8 __attribute__((ext_vector_type(8)));
template <int P>
__global__ void __launch_bounds__(512, 2) mfma_loop_f8(const i32x8* __restrict__ src, float* __restrict__ out, int iters) {
  const int lane = threadIdx.x & 63;
  i32x8 a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = src[(i * 64 + lane) % 512];
    b[i] = src[((i + 4) * 64 + lane) % 512];
  }
  float s = 0.f;
  if constexpr (P == 7) {
    f32x16 acc[4] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 32; ++j)
        acc[j & 3] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[j & 3], b[(j >> 2) & 3], acc[j & 3], 0, 0, 0, 0, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) s += acc[c][r];
  } else {
    f32x4 acc[16] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 64; ++j)
        acc[j & 15] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[j & 3], b[(j >> 1) & 3], acc[j & 15], 0, 0, 0, 0, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < 16; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) s += acc[c][r];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int P>
double run_f8(const i32x8* src, float* out, int iters) {
  const int grid = 256 * 2, block = 512;
  hipLaunchKernelGGL(mfma_loop_f8<P>, dim3(grid), dim3(block), 0, 0, src, out, 10);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma_loop_f8<P>, dim3(grid), dim3(block), 0, 0, src, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  // per iteration and wave: 32 x (32 x 32 x 64) or 64 x (16 x 16 x 128) MACs = the same 2^21
  const double flop = 2.0 * 32 * 32 * 64 * 32.0 * iters * (grid * block / 64);
  return flop / (ms * 1e-3) / 1e12;
}

template <int P>
double run(const bf16x8* src, float* out, int iters) {
  const int grid = 256 * 2, block = 512;
  if constexpr (P >= 5) hipLaunchKernelGGL(mfma_loop16<P>, dim3(grid), dim3(block), 0, 0, src, out, 10);
  else hipLaunchKernelGGL(mfma_loop<P>, dim3(grid), dim3(block), 0, 0, src, out, 10);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  if constexpr (P >= 5) hipLaunchKernelGGL(mfma_loop16<P>, dim3(grid), dim3(block), 0, 0, src, out, iters);
  else hipLaunchKernelGGL(mfma_loop<P>, dim3(grid), dim3(block), 0, 0, src, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = 2.0 * 32 * 32 * 16 * 64.0 * iters * (grid * block / 64);
  return flop / (ms * 1e-3) / 1e12;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  std::vector<unsigned short> h(1024 * 8);
  unsigned x = 12345u;
  for (auto& v : h) {  // random bf16 of moderate magnitude: sign, exponent 120..133, random mantissa
    x = x * 1664525u + 1013904223u;
    v = (unsigned short)(((x >> 31) << 15) | (((x >> 20) % 14 + 120) << 7) | ((x >> 8) & 127));
  }
  bf16x8 *src, *zsrc;
  float* out;
  hipMalloc(&src, h.size() * 2);
  hipMalloc(&zsrc, h.size() * 2);
  hipMalloc(&out, 256 * 2 * 512 * 4);
  hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  hipMemset(zsrc, 0, h.size() * 2);
  // random e4m3 bytes (finite: exponent field below 15 keeps clear of NaN), 512 lanes x 32 B
  std::vector<unsigned char> h8(512 * 32);
  for (auto& v : h8) {
    x = x * 1664525u + 1013904223u;
    v = (unsigned char)(((x >> 31) << 7) | ((((x >> 20) % 6) + 4) << 3) | ((x >> 8) & 7));
  }
  void* src8;
  hipMalloc(&src8, h8.size());
  hipMemcpy(src8, h8.data(), h8.size(), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    printf("pattern 0 (A, B change every MFMA): %.1f TFLOP/s\n", run<0>(src, out, iters));
    printf("pattern 1 (A every MFMA, B every 8): %.1f TFLOP/s\n", run<1>(src, out, iters));
    printf("pattern 2 (A every 8, B every MFMA): %.1f TFLOP/s\n", run<2>(src, out, iters));
    printf("pattern 3 (A, B fixed): %.1f TFLOP/s\n", run<3>(src, out, iters));
    printf("pattern 4 (pattern 0, zero data): %.1f TFLOP/s\n", run<4>(zsrc, out, iters));
    printf("pattern 5 (16x16x32, A, B change every MFMA): %.1f TFLOP/s\n", run<5>(src, out, iters));
    printf("pattern 6 (16x16x32, zero data): %.1f TFLOP/s\n", run<6>(zsrc, out, iters));
    printf("pattern 0 again: %.1f TFLOP/s\n", run<0>(src, out, iters));
    printf("pattern 7 (fp8 32x32x64, random): %.1f TFLOP/s\n", run_f8<7>((const i32x8*)src8, out, iters));
    printf("pattern 8 (fp8 16x16x128, random): %.1f TFLOP/s\n", run_f8<8>((const i32x8*)src8, out, iters));
    printf("pattern 7z (fp8 32x32x64, zeros): %.1f TFLOP/s\n", run_f8<7>((const i32x8*)zsrc, out, iters));
    printf("pattern 8z (fp8 16x16x128, zeros): %.1f TFLOP/s\n", run_f8<8>((const i32x8*)zsrc, out, iters));
    fflush(stdout);
  }
  return 0;
}
