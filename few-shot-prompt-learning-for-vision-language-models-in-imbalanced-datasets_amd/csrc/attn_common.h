// Device helpers shared by the attention kernels (attention.hip, attention_prefix.hip):
// 64-wide head rows, 16-bit MFMA tile operands, ds_read_b64_tr_b16 transposed LDS reads.
#pragma once
#include "common.h"

namespace clipk {

constexpr float kScale = 0.125f;  // 1/sqrt(64)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ void load_row64(const T* p, float* out) {
  constexpr int V = Vec16<T>::N;
#pragma unroll
  for (int c = 0; c < 64 / V; ++c) load16_f32<T>(p + c * V, out + c * V);
}

template <typename T>
__device__ __forceinline__ void store_row64(T* p, const float* in) {
  constexpr int V = Vec16<T>::N;
#pragma unroll
  for (int c = 0; c < 64 / V; ++c) store16_f32<T>(p + c * V, in + c * V);
}

__device__ __forceinline__ float dot64(const float* a, const float* b) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
  for (int d = 0; d < 64; d += 4) {
    s0 = fmaf(a[d], b[d], s0);
    s1 = fmaf(a[d + 1], b[d + 1], s1);
    s2 = fmaf(a[d + 2], b[d + 2], s2);
    s3 = fmaf(a[d + 3], b[d + 3], s3);
  }
  return (s0 + s1) + (s2 + s3);
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
constexpr int TRS = 72;  // LDS row stride in 16-bit elements (64 + 8 pad, 8-byte aligned)

__device__ __forceinline__ s16x8 ld_row16(const void* p, bool ok) {
  if (!ok) return (s16x8){0, 0, 0, 0, 0, 0, 0, 0};
  return *reinterpret_cast<const s16x8*>(p);
}

// convert 8 elements of T (raw 16 B) to bf16 bits
template <typename T>
__device__ __forceinline__ s16x8 to_bf16x8(s16x8 v) {
  if constexpr (__is_same(T, bf16)) {
    return v;
  } else {
    f16x8 h = __builtin_bit_cast(f16x8, v);
    bf16x8 b;
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = (bf16)(float)h[i];
    return __builtin_bit_cast(s16x8, b);
  }
}

__device__ __forceinline__ f32x4 mfma32_bf16(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16_bf16(s16x4 a, s16x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ s16x4 pack_bf16x4(float a, float b, float c, float d) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  bf16x4 v = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
  return __builtin_bit_cast(s16x4, v);
}
__device__ __forceinline__ s16x4 tr_read(const short* tile, int rbase, int cbase, int lane) {
  const int li = lane & 15;
  const short* p = tile + (rbase + (li >> 2)) * TRS + cbase + 4 * (li & 3);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
}

template <typename T>
__device__ __forceinline__ f32x4 mfma32_t(s16x8 a, s16x8 b, f32x4 c) {
  if constexpr (__is_same(T, f16))
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
template <typename T>
__device__ __forceinline__ f32x4 mfma16_t(s16x4 a, s16x4 b, f32x4 c) {
  if constexpr (__is_same(T, f16)) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(h4, a), __builtin_bit_cast(h4, b), c, 0, 0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
  }
}
template <typename T>
__device__ __forceinline__ s16x4 pack4(float a, float b, float c, float d) {
  typedef T t4 __attribute__((ext_vector_type(4)));
  t4 v = {(T)a, (T)b, (T)c, (T)d};
  return __builtin_bit_cast(s16x4, v);
}

}  // namespace clipk
