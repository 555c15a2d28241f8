// MFMA throughput yardstick (not part of libclipk.so): back-to-back v_mfma_f32_16x16x32_f16 on
// register operands (random data passed in), one or two waves per SIMD, every CU busy -- the
// rate the chip sustains under its clock management, against which the GEMM kernels' fractions
// of the 2.5 PF nominal peak can be read. Also the in-kernel clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int WPS>
__global__ __launch_bounds__(256 * WPS, 1) void mfma_loop(const f16x8* __restrict__ src, float* out, int iters,
                                                          unsigned long long* clk) {
  const int t = threadIdx.x;
  f16x8 a = src[t & 255], b = src[(t + 7) & 255];
  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[i], 0, 0, 0);
    a[0] += (f16)1e-3f;  // keep the loop from being hoisted
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + t] = s;
  if (t == 0 && blockIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
}

extern "C" int mfma_peak(int wps, const void* src, void* out, int iters, int blocks, void* clk, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (wps == 1)
    hipLaunchKernelGGL((mfma_loop<1>), dim3(blocks), dim3(256), 0, st, (const f16x8*)src, (float*)out, iters,
                       (unsigned long long*)clk);
  else
    hipLaunchKernelGGL((mfma_loop<2>), dim3(blocks), dim3(512), 0, st, (const f16x8*)src, (float*)out, iters,
                       (unsigned long long*)clk);
  return (int)hipGetLastError();
}
