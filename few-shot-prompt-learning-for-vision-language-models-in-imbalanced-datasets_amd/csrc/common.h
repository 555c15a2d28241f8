// Shared device helpers for the gfx950 (CDNA4) CoOp/CoCoOp kernels.
// Written for wave64 / MFMA only: no CUDA shims, no dual-platform paths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/clipk.h"

typedef _Float16 f16;
typedef __bf16 bf16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define CLIPK_LDS_ALIGN __attribute__((aligned(16)))

namespace clipk {

constexpr int kWave = 64;

// GEMM input tag of the split-fp16 fp32-class path (CLIPK_F32S): A fp32, B split-packed
// (clipk_split_pack); 4 bytes per element on both operands.
struct f32s { float v; };
// ... and CLIPK_F32S16: the same operands, B's lo parts all zero (the weight-lo product skipped)
struct f32h { float v; };
template <typename T> constexpr bool is_split_v = __is_same(T, f32s) || __is_same(T, f32h);

template <typename T> struct DT;
template <> struct DT<float> { static constexpr int id = CLIPK_F32; };
template <> struct DT<f16>   { static constexpr int id = CLIPK_F16; };
template <> struct DT<bf16>  { static constexpr int id = CLIPK_BF16; };
template <> struct DT<f32s>  { static constexpr int id = CLIPK_F32S; };
template <> struct DT<f32h>  { static constexpr int id = CLIPK_F32S16; };

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(f16 x) { return (float)x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }

template <typename T> __device__ __forceinline__ T from_f32(float x) { return (T)x; }

// 16 bytes of T -> fp32 values (8 for 16-bit types, 4 for fp32).
template <typename T> struct Vec16 {
  static constexpr int N = 16 / sizeof(T);
};

// Load N=16/sizeof(T) elements as fp32 from a 16-byte aligned address.
template <typename T>
__device__ __forceinline__ void load16_f32(const T* p, float* out) {
  if constexpr (sizeof(T) == 4) {
    f32x4 v = *reinterpret_cast<const f32x4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = v[i];
  } else {
    typedef T t8 __attribute__((ext_vector_type(8)));
    t8 v = *reinterpret_cast<const t8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = (float)v[i];
  }
}

template <typename T>
__device__ __forceinline__ void store16_f32(T* p, const float* in) {
  if constexpr (sizeof(T) == 4) {
    f32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = in[i];
    *reinterpret_cast<f32x4*>(p) = v;
  } else {
    typedef T t8 __attribute__((ext_vector_type(8)));
    t8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (T)in[i];
    *reinterpret_cast<t8*>(p) = v;
  }
}

// 4 consecutive elements (fp32 in registers) -> memory of type T.
template <typename T>
__device__ __forceinline__ void store4(T* p, float a, float b, float c, float d) {
  if constexpr (sizeof(T) == 4) {
    f32x4 v = {a, b, c, d};
    *reinterpret_cast<f32x4*>(p) = v;
  } else {
    typedef T t4 __attribute__((ext_vector_type(4)));
    t4 v = {(T)a, (T)b, (T)c, (T)d};
    *reinterpret_cast<t4*>(p) = v;
  }
}

template <typename T>
__device__ __forceinline__ void load4(const T* p, float* o) {
  if constexpr (sizeof(T) == 4) {
    f32x4 v = *reinterpret_cast<const f32x4*>(p);
    o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = v[3];
  } else {
    typedef T t4 __attribute__((ext_vector_type(4)));
    t4 v = *reinterpret_cast<const t4*>(p);
    o[0] = (float)v[0]; o[1] = (float)v[1]; o[2] = (float)v[2]; o[3] = (float)v[3];
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Reductions inside aligned groups of G lanes (G power of two <= 64).
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int G>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = G / 2; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// QuickGELU (PromptSRC/clip/model.py:162-164): x * sigmoid(1.702 x), and its derivative.
// v_exp_f32 + v_rcp_f32 (1 ulp) instead of an IEEE division: these run per output element
// in the GEMM epilogues, where a full-precision divide costed ~10 VALU instructions. The
// exponent is formed with ONE multiply (-1.702 * log2 e folded) straight into v_exp_f32
// (exp2): __expf(-1.702f * x) emitted two v_mul_f32 per element.
constexpr float kQgeluExp2 = -2.4554669595930157f;  // -1.702 * log2(e)
__device__ __forceinline__ float qgelu_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(kQgeluExp2 * x));
}
__device__ __forceinline__ float quick_gelu(float x) { return x * qgelu_sigmoid(x); }
__device__ __forceinline__ float quick_gelu_grad(float x) {
  const float s = qgelu_sigmoid(x);
  return s * fmaf(1.702f * x, 1.0f - s, 1.0f);  // s + 1.702 x s (1 - s)
}

// The lo parts of a split (hi = fp16(x), lo = fp16(x - hi)) of 4 fp32 values whose hi parts are
// the fp16 pairs h01 = (x0, x1), h23 = (x2, x3): v_fma_mix forms x - hi exactly in fp32 and
// rounds once, bitwise (_Float16)(x - (float)hi), in 4 instructions instead of cvt + sub + cvt
// per value. Consumers must not be MFMA operands without their own wait states (gemm_kernel.h
// split_lo8 carries them for that case).
__device__ __forceinline__ void split_lo4(float x0, float x1, float x2, float x3, unsigned h01, unsigned h23,
                                          unsigned& l01, unsigned& l23) {
  asm("v_fma_mixlo_f16 %0, %2, 1.0, -%6 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %3, 1.0, -%6 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %1, %4, 1.0, -%7 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %5, 1.0, -%7 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(l01), "=&v"(l23)
      : "v"(x0), "v"(x1), "v"(x2), "v"(x3), "v"(h01), "v"(h23));
}

}  // namespace clipk

#define CLIPK_CHECK_LAUNCH()                                  \
  do {                                                        \
    hipError_t _e = hipGetLastError();                        \
    if (_e != hipSuccess) return (int)_e;                     \
  } while (0)
