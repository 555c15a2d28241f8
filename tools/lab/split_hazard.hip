// What wait states hipcc's gfx950 hazard recognizer puts between the split's VALU writes and an
// MFMA reading them, when the sequence is compiler-visible (the reference for the inline-asm
// split in gemm_kernel.h split_lo8, which must carry them itself). Build for inspection only:
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -S -o - tools/lab/split_hazard.hip
// (-fno-slp-vectorize keeps the scalar fma -> v_fma_mixlo/hi_f16 selection; with SLP on, hipcc
// packs the FMAs into v_pk_fma_f32 + v_cvt_pk_f16_f32 and pads that VALU -> MFMA pair the same way.)
#include <hip/hip_runtime.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// lo = fp16(a * m - f32(h)): v_fma_mixlo / v_fma_mixhi writing the MFMA's B operand
extern "C" __global__ void mix_then_mfma(const float* a, const float* m, const _Float16* h, const f16x8* A,
                                         f32x4* out) {
  const int i = threadIdx.x;
  f16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (_Float16)__builtin_fmaf(a[8 * i + j], m[8 * i + j], -(float)h[8 * i + j]);
  out[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[i], v, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
}
