// Device helpers shared by the attention kernels (attention.hip, attention_prefix.hip):
// 64-wide head rows, 16-bit MFMA tile operands, ds_read_b64_tr_b16 transposed LDS reads.
#pragma once
#include "common.h"

#ifndef CLIPK_ATTN_SNT
#define CLIPK_ATTN_SNT 0
#endif

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

// 8 consecutive columns of a row as fp32 (one 16-B load for 16-bit T, two for fp32)
template <typename T>
__device__ __forceinline__ void load_cols8(const T* p, float* out) {
  constexpr int V = Vec16<T>::N;
#pragma unroll
  for (int c = 0; c < 8 / V; ++c) load16_f32<T>(p + c * V, out + c * V);
}

__device__ __forceinline__ void lds_fence_a() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

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

// fp32 kernels with lane = 4 * row + 16-column slice: quad sums, 16-float row slices
__device__ __forceinline__ float quad_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
}
__device__ __forceinline__ void ld16(const float* __restrict__ p, float* v) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const f32x4 t = reinterpret_cast<const f32x4*>(p)[c];
    v[4 * c] = t[0]; v[4 * c + 1] = t[1]; v[4 * c + 2] = t[2]; v[4 * c + 3] = t[3];
  }
}
__device__ __forceinline__ void st16(float* __restrict__ p, const float* v) {
#pragma unroll
  for (int c = 0; c < 4; ++c)
    reinterpret_cast<f32x4*>(p)[c] = (f32x4){v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]};
}
// lane slice s of a 64-float head row: columns {kCs c + kSl s + e : c, e < 4}. Interleaved
// (CLIPK_F32_IL=1, default): each f32x4 load of the 4 lanes of a row covers 64 contiguous
// bytes; contiguous (0): lane s holds columns 16 s .. 16 s + 15. Every global and LDS row
// access of the fp32 attention kernels uses this one map, so q / k / v / dO / o slices pair up.
#ifndef CLIPK_F32_IL
#define CLIPK_F32_IL 1
#endif
constexpr int kSl = CLIPK_F32_IL ? 4 : 16, kCs = CLIPK_F32_IL ? 16 : 4;
__device__ __forceinline__ void ld16x(const float* __restrict__ p, float* v) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const f32x4 t = *reinterpret_cast<const f32x4*>(p + kCs * c);
    v[4 * c] = t[0]; v[4 * c + 1] = t[1]; v[4 * c + 2] = t[2]; v[4 * c + 3] = t[3];
  }
}
__device__ __forceinline__ void st16x(float* __restrict__ p, const float* v) {
#pragma unroll
  for (int c = 0; c < 4; ++c)
    *reinterpret_cast<f32x4*>(p + kCs * c) = (f32x4){v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]};
}
// The parts of one fp32 value as a split GEMM forms them (gemm_kernel.h split8): hi = fp16(x),
// lo = fp16(x - hi), of the ROUNDED x (opaque copy: no contraction with x's producing arithmetic)
__device__ __forceinline__ void split_parts(float v, _Float16& hi, _Float16& lo) {
  float x = v;
  asm volatile("" : "+v"(x));
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}
// st16x in the pre-split operand form of a split GEMM's A (include/clipk.h CLIPK_A_SPLIT: per 8
// consecutive columns 16 B of hi parts then 16 B of lo parts, 4 B per element as the fp32 row).
// Called by all 4 lanes of a row (lane = 4 r + s, the slice map above, interleaved only): chunk c
// of lanes s = 2j, 2j + 1 is the 8-column group 2c + j, so the pair trades halves over one DPP
// quad_perm [1,0,3,2] -- the even lane sends its lo parts and gets its partner's hi parts -- and
// each lane stores one whole 16-B half (even: the group's hi parts, odd: its lo parts), the store
// count of st16x. The lo parts are v_fma_mix, as gemm_kernel.h split_lo8 (their consumers here
// are a VALU select and a store: no MFMA reads them, so no wait states in the statement).
static_assert(CLIPK_F32_IL, "st16x_split: the interleaved slice map");
__device__ __forceinline__ void st16x_split(float* __restrict__ p, const float* v, int s) {
  const bool odd = s & 1;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float x[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[e] = v[4 * c + e];
      asm volatile("" : "+v"(x[e]));  // the rounded fp32 value (no contraction with its producer)
    }
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const unsigned h0 = __builtin_bit_cast(unsigned, (h2){(_Float16)x[0], (_Float16)x[1]});
    const unsigned h1 = __builtin_bit_cast(unsigned, (h2){(_Float16)x[2], (_Float16)x[3]});
    unsigned l0, l1;
    split_lo4(x[0], x[1], x[2], x[3], h0, h1, l0, l1);
    const unsigned s0 = odd ? h0 : l0, s1 = odd ? h1 : l1;  // the half the partner stores
    const unsigned y0 = (unsigned)__builtin_amdgcn_mov_dpp((int)s0, 0xB1, 0xF, 0xF, false);
    const unsigned y1 = (unsigned)__builtin_amdgcn_mov_dpp((int)s1, 0xB1, 0xF, 0xF, false);
    const uintptr_t a = reinterpret_cast<uintptr_t>(p + kCs * c);
    uint4* grp = reinterpret_cast<uint4*>(a & ~uintptr_t(31));
    // even: hi parts (own columns 0-3, partner's 4-7); odd: lo parts (partner's 0-3, own 4-7)
    grp[odd] = odd ? (uint4){y0, y1, l0, l1} : (uint4){h0, h1, y0, y1};
  }
}

__device__ __forceinline__ float dot16(const float* a, const float* b) {
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int d = 0; d < 16; d += 2) {
    s0 = fmaf(a[d], b[d], s0);
    s1 = fmaf(a[d + 1], b[d + 1], s1);
  }
  return s0 + s1;
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

// convert 8 elements of T (raw 16 B) to the math type TG (the backward's grad dtype)
template <typename T, typename TG>
__device__ __forceinline__ s16x8 to_g8(s16x8 v) {
  if constexpr (__is_same(T, TG)) {
    return v;
  } else if constexpr (__is_same(TG, bf16)) {
    return to_bf16x8<T>(v);
  } else {
    bf16x8 b = __builtin_bit_cast(bf16x8, v);
    f16x8 h;
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = (f16)(float)b[i];
    return __builtin_bit_cast(s16x8, h);
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

// Reductions over lane bits 4 and 5 (the four 16-lane rows of an MFMA 16x16 tile) by
// v_permlane32_swap / v_permlane16_swap: VALU only (a __shfl_xor is an LDS ds_bpermute round
// trip), and every lane ends with the same value (the adds are the same pairs in the same order).
__device__ __forceinline__ float xmax4(float v) {  // max over lane bits 4 and 5
  auto a = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false,
                                            false);
  v = fmaxf(__builtin_bit_cast(float, (unsigned)a[0]), __builtin_bit_cast(float, (unsigned)a[1]));
  auto b = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false,
                                            false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)b[0]), __builtin_bit_cast(float, (unsigned)b[1]));
}
__device__ __forceinline__ float xsum4(float v) {  // sum over lane bits 4 and 5
  auto a = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false,
                                            false);
  v = __builtin_bit_cast(float, (unsigned)a[0]) + __builtin_bit_cast(float, (unsigned)a[1]);
  auto b = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false,
                                            false);
  return __builtin_bit_cast(float, (unsigned)b[0]) + __builtin_bit_cast(float, (unsigned)b[1]);
}


// Store a 16-row x 64-column (one head) tile held in the MFMA accumulator layout -- lane
// (r16, g4) holds row r16, columns 16t + 4g4 .. +3 in o[t] -- as 16-bit values. The packed
// values go through a lane/slot butterfly (v_permlane32_swap: lane bit 5 <-> slot bit 0, then
// v_permlane16_swap: lane bit 4 <-> slot bit 0) that leaves lane g4 holding columns
// 8g4 .. 8g4+7 and 32+8g4 .. +7, so a row leaves as two 16-B stores per lane (each store
// instruction: 16 rows x 64 contiguous bytes) instead of four 8-B ones. Every lane of the
// wave must execute it (the swaps cross lanes); `ok` masks only the stores.
template <typename T>
__device__ __forceinline__ void store_tile64(T* rowp, const f32x4 (&o)[4], float scale, bool ok) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  uint32_t d[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const u32x2 u = __builtin_bit_cast(u32x2, pack4<T>(o[t][0] * scale, o[t][1] * scale, o[t][2] * scale,
                                                       o[t][3] * scale));
    d[t][0] = u[0];
    d[t][1] = u[1];
  }
#pragma unroll
  for (int s = 0; s < 4; s += 2)
#pragma unroll
    for (int dw = 0; dw < 2; ++dw) {
      const auto r = __builtin_amdgcn_permlane32_swap(d[s][dw], d[s + 1][dw], false, false);
      d[s][dw] = r[0];
      d[s + 1][dw] = r[1];
    }
#pragma unroll
  for (int s = 0; s < 4; s += 2)
#pragma unroll
    for (int dw = 0; dw < 2; ++dw) {
      const auto r = __builtin_amdgcn_permlane16_swap(d[s][dw], d[s + 1][dw], false, false);
      d[s][dw] = r[0];
      d[s + 1][dw] = r[1];
    }
  if (ok) {
    const int g4 = (threadIdx.x & 63) >> 4;
#if CLIPK_ATTN_SNT  // build-time A/B knob: non-temporal output stores
    __builtin_nontemporal_store((u32x4){d[0][0], d[0][1], d[1][0], d[1][1]}, reinterpret_cast<u32x4*>(rowp + 8 * g4));
    __builtin_nontemporal_store((u32x4){d[2][0], d[2][1], d[3][0], d[3][1]},
                                reinterpret_cast<u32x4*>(rowp + 32 + 8 * g4));
#else
    *reinterpret_cast<u32x4*>(rowp + 8 * g4) = (u32x4){d[0][0], d[0][1], d[1][0], d[1][1]};
    *reinterpret_cast<u32x4*>(rowp + 32 + 8 * g4) = (u32x4){d[2][0], d[2][1], d[3][0], d[3][1]};
#endif
  }
}

}  // namespace clipk
