// LayerNorm forward / input-grad backward as wavefront row reductions (HBM-bound).
// Reference: PromptSRC/clip/model.py:153-159 (fp32 upcast, eps 1e-5, affine).
// One wave per CLIPK_LN_RPW rows, each row kept in registers (width <= 1024), two-pass mean/variance from
// registers (no E[x^2]-E[x]^2 cancellation); 8 consecutive elements per lane (16-B accesses
// of 16-bit rows) when the width is a multiple of 512, else 4. The input row (the residual
// stream) is fp32 or, for the 16-bit text residual stream, the activation dtype (statistics
// always in fp32). Optional row gather (in_rows) for ln_final on EOT rows and ln_post on
// CLS rows, optional scatter (out_rows) on the backward.
#include <type_traits>

#include "common.h"

namespace clipk {

constexpr int LN_MAXV = 4;  // 4-element vectors per lane -> width <= 1024

// VW consecutive elements per lane per chunk: 8 (16-B loads of 16-bit rows, 2x16-B of fp32)
// when width is a multiple of 512, else 4; NC chunks cover width <= 1024.
// Cache policy knobs (build-time A/B, tools/ab_bench.sh): CLIPK_LN_NT bit 0 = non-temporal
// row loads, bit 1 = non-temporal stores (16-bit rows).
#ifndef CLIPK_LN_NT
#define CLIPK_LN_NT 0
#endif
template <typename T, int VW>
__device__ __forceinline__ void ldv(const T* p, float* o) {
  if constexpr (VW == 4) {
    load4<T>(p, o);
  } else if constexpr (sizeof(T) == 2) {
#if CLIPK_LN_NT & 1
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    typedef T t8 __attribute__((ext_vector_type(8)));
    const t8 v = __builtin_bit_cast(t8, __builtin_nontemporal_load(reinterpret_cast<const u4*>(p)));
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)v[i];
#else
    load16_f32<T>(p, o);
#endif
  } else {
    load16_f32<T>(p, o);
    load16_f32<T>(p + 4, o + 4);
  }
}
template <typename T, int VW>
__device__ __forceinline__ void stv(T* p, const float* v) {
  if constexpr (__is_same(T, f32s)) {
    // the pre-split operand form of a split GEMM's A (include/clipk.h CLIPK_A_SPLIT): per 8
    // consecutive elements 16 B of fp16 hi = fp16(v) then 16 B of lo = fp16(v - hi), of the
    // ROUNDED fp32 v (opaque copy: no contraction with v's producing arithmetic). VW 8 = one whole
    // group; VW 4 = half a group (hi and lo 8 B each, 16 B apart).
    float x[VW];
#pragma unroll
    for (int i = 0; i < VW; ++i) {
      x[i] = v[i];
      asm volatile("" : "+v"(x[i]));
    }
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    h4 hi[VW / 4], lo[VW / 4];
#pragma unroll
    for (int i = 0; i < VW; ++i) {
      hi[i / 4][i % 4] = (_Float16)x[i];
      lo[i / 4][i % 4] = (_Float16)(x[i] - (float)hi[i / 4][i % 4]);
    }
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);  // element offset within its 8-group: 0 or 4
    char* g = reinterpret_cast<char*>(a & ~uintptr_t(31));
    const int half = (int)((a >> 4) & 1);
    if constexpr (VW == 8) {
      *reinterpret_cast<uint4*>(g) = __builtin_bit_cast(uint4, (f16x8){hi[0][0], hi[0][1], hi[0][2], hi[0][3],
                                                                       hi[1][0], hi[1][1], hi[1][2], hi[1][3]});
      *reinterpret_cast<uint4*>(g + 16) = __builtin_bit_cast(uint4, (f16x8){lo[0][0], lo[0][1], lo[0][2], lo[0][3],
                                                                            lo[1][0], lo[1][1], lo[1][2], lo[1][3]});
    } else {
      *reinterpret_cast<uint2*>(g + 8 * half) = __builtin_bit_cast(uint2, hi[0]);
      *reinterpret_cast<uint2*>(g + 16 + 8 * half) = __builtin_bit_cast(uint2, lo[0]);
    }
  } else if constexpr (VW == 4) {
    store4<T>(p, v[0], v[1], v[2], v[3]);
  } else if constexpr (sizeof(T) == 2) {
#if CLIPK_LN_NT & 2
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    typedef T t8 __attribute__((ext_vector_type(8)));
    t8 h;
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = (T)v[i];
    __builtin_nontemporal_store(__builtin_bit_cast(u4, h), reinterpret_cast<u4*>(p));
#else
    store16_f32<T>(p, v);
#endif
  } else {
    store16_f32<T>(p, v);
    store16_f32<T>(p + 4, v + 4);
  }
}

// RPW rows per wave: every row's loads are issued before the first reduction, so a wave keeps
// RPW rows of HBM traffic in flight; gamma / beta loaded once per wave. NC = 64-lane chunks per
// row (width / VW / 64 rounded up). The per-row arithmetic does not depend on RPW. Same-box A/B
// (profiles/r02p_ab_ln_rpw.txt, headline step): forward 1 -> 2 rows per wave 0.52 -> 0.50
// ms/step, 4 rows 0.58; backward 1 row 0.79, 2 rows 0.85, 4 rows 1.06 (its three row streams
// per row already keep the memory system busy at one row per wave).
#ifndef CLIPK_LN_RPW
#define CLIPK_LN_RPW 2
#endif
#ifndef CLIPK_LN_RPW_BWD
#define CLIPK_LN_RPW_BWD 1
#endif
template <typename TI, typename TO, int VW, int NC, int RPW>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int rows, int width, const TI* __restrict__ x,
                                                     int ldx, const int* __restrict__ in_rows,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, TO* __restrict__ out,
                                                     int ldo, float* __restrict__ mean,
                                                     float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int r0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (r0 >= rows) return;
  const int nv = width / VW;  // vectors per row
  float v[RPW][NC][VW], gg[NC][VW], bb[NC][VW];
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    const int r = min(r0 + j, rows - 1);  // rows past the end: a valid row, never stored
    const TI* xp = x + (size_t)(in_rows ? in_rows[r] : r) * ldx;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = lane + i * 64;
      if (c < nv) {
        ldv<TI, VW>(xp + c * VW, v[j][i]);
      } else {
#pragma unroll
        for (int k = 0; k < VW; ++k) v[j][i][k] = 0.f;
      }
    }
  }
  // gamma / beta are issued with x: loaded after the reductions they were one more dependent
  // round trip per row
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + i * 64;
    if (c < nv) {
      ldv<float, VW>(gamma + c * VW, gg[i]);
      ldv<float, VW>(beta + c * VW, bb[i]);
    }
  }
  const float inv_w = 1.0f / (float)width;
  float mu[RPW], rs[RPW];
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i)
#pragma unroll
      for (int k = 0; k < VW; ++k) s += v[j][i][k];
    mu[j] = wave_sum(s) * inv_w;
  }
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = lane + i * 64;
      if (c < nv) {
#pragma unroll
        for (int k = 0; k < VW; ++k) { const float d = v[j][i][k] - mu[j]; q += d * d; }
      }
    }
    rs[j] = rsqrtf(wave_sum(q) * inv_w + 1e-5f);
  }
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    const int r = r0 + j;
    if (r >= rows) break;
    TO* op = out + (size_t)r * ldo;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = lane + i * 64;
      if (c < nv) {
        float o[VW];
#pragma unroll
        for (int k = 0; k < VW; ++k) o[k] = (v[j][i][k] - mu[j]) * rs[j] * gg[i][k] + bb[i][k];
        stv<TO, VW>(op + c * VW, o);
      }
    }
    if (lane == 0) {
      if (mean) mean[r] = mu[j];
      if (rstd) rstd[r] = rs[j];
    }
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) + dres,   g = dy * gamma
// RL: the incoming residual gradient dres is in the low-precision dtype TL (a 16-bit residual-
// gradient stream, updated in place: dres == dx_lp is allowed, each lane reads its chunk
// before writing it); dx (fp32) may then be null.
template <typename TL, typename TD, typename TX, int VW, bool RL, int NC, int RPW>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int rows, int width, const TD* __restrict__ dy,
                                                     int lddy, const TX* __restrict__ x, int ldx,
                                                     const int* __restrict__ x_rows,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd,
                                                     const void* dres_v, int lddres,
                                                     float* __restrict__ dx, TL* dx_lp,
                                                     const int* __restrict__ out_rows, int ldo) {
  const int lane = threadIdx.x & 63;
  const int r0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (r0 >= rows) return;
  const int nv = width / VW;
  typedef typename std::conditional<RL, TL, float>::type TR;
  float xv[RPW][NC][VW], dv[RPW][NC][VW], rv[RPW][NC][VW], gg[NC][VW];
  int orow[RPW];
  float mu[RPW], rs[RPW];
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    const int r = min(r0 + j, rows - 1);  // rows past the end: loaded, never stored
    orow[j] = out_rows ? out_rows[r] : r;
    mu[j] = mean[r];
    rs[j] = rstd[r];
    const TX* xp = x + (size_t)(x_rows ? x_rows[r] : r) * ldx;
    const TD* dp = dy + (size_t)r * lddy;
    const TR* rp = dres_v ? (const TR*)dres_v + (size_t)orow[j] * lddres : nullptr;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = lane + i * 64;
      if (c < nv) {
        ldv<TX, VW>(xp + c * VW, xv[j][i]);
        ldv<TD, VW>(dp + c * VW, dv[j][i]);
        // the residual gradient is issued with the other operands (not after the reductions)
        if (rp) ldv<TR, VW>(rp + c * VW, rv[j][i]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + i * 64;
    if (c < nv) ldv<float, VW>(gamma + c * VW, gg[i]);
  }
  const float inv_w = 1.0f / (float)width;
  float m1[RPW], m2[RPW];
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = lane + i * 64;
      if (c < nv) {
#pragma unroll
        for (int k = 0; k < VW; ++k) {
          xv[j][i][k] = (xv[j][i][k] - mu[j]) * rs[j];  // xhat
          dv[j][i][k] = dv[j][i][k] * gg[i][k];         // g = dy * gamma
          s1 += dv[j][i][k];
          s2 += dv[j][i][k] * xv[j][i][k];
        }
      }
    }
    m1[j] = wave_sum(s1) * inv_w;
    m2[j] = wave_sum(s2) * inv_w;
  }
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    if (r0 + j >= rows) break;
    const bool has_r = dres_v != nullptr;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = lane + i * 64;
      if (c < nv) {
        float o[VW];
#pragma unroll
        for (int k = 0; k < VW; ++k) o[k] = rs[j] * (dv[j][i][k] - m1[j] - xv[j][i][k] * m2[j]);
        if (has_r) {
#pragma unroll
          for (int k = 0; k < VW; ++k) o[k] += rv[j][i][k];
        }
        if (dx) stv<float, VW>(dx + (size_t)orow[j] * ldo + c * VW, o);
        if (dx_lp) stv<TL, VW>(dx_lp + (size_t)orow[j] * ldo + c * VW, o);
      }
    }
  }
}

}  // namespace clipk

using namespace clipk;

template <typename TI, int RPW>
static int ln_fwd_launch_rpw(int out_dtype, int rows, int width, const TI* x, int ldx, const int* in_rows,
                             const float* gamma, const float* beta, void* out, int ldo, float* mean, float* rstd,
                             hipStream_t st) {
  dim3 grid((rows + 4 * RPW - 1) / (4 * RPW)), block(256);
  const bool v8 = width % 512 == 0 && ldx % 8 == 0 && ldo % 8 == 0;
  const bool one = v8 && width == 512;  // one 64-lane chunk of 8 elements per row
#define CLIPK_LNF(TOUT)                                                                                        \
  if (one)                                                                                                     \
    hipLaunchKernelGGL((ln_fwd_kernel<TI, TOUT, 8, 1, RPW>), grid, block, 0, st, rows, width, x, ldx, in_rows, \
                       gamma, beta, (TOUT*)out, ldo, mean, rstd);                                              \
  else if (v8)                                                                                                 \
    hipLaunchKernelGGL((ln_fwd_kernel<TI, TOUT, 8, 2, RPW>), grid, block, 0, st, rows, width, x, ldx, in_rows, \
                       gamma, beta, (TOUT*)out, ldo, mean, rstd);                                              \
  else                                                                                                         \
    hipLaunchKernelGGL((ln_fwd_kernel<TI, TOUT, 4, 4, RPW>), grid, block, 0, st, rows, width, x, ldx, in_rows, \
                       gamma, beta, (TOUT*)out, ldo, mean, rstd);
  switch (out_dtype) {
    case CLIPK_F32: CLIPK_LNF(float) break;
    case CLIPK_F16: CLIPK_LNF(f16) break;
    case CLIPK_BF16: CLIPK_LNF(bf16) break;
    default: return CLIPK_EDTYPE;
  }
#undef CLIPK_LNF
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}
// Rows per wave: CLIPK_LN_RPW (2) for the 16-bit residual stream; for an fp32 one (PREC fp32 /
// fp32s: twice the bytes per row) knob CLIPK_LN_RPW32 = 1, 2 or 4 (default 2)
static int ln_rpw32() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLIPK_LN_RPW32");
    v = e ? atoi(e) : 2;
    if (v != 1 && v != 4) v = 2;
  }
  return v;
}
template <typename TI>
static int ln_fwd_launch(int out_dtype, int rows, int width, const TI* x, int ldx, const int* in_rows,
                         const float* gamma, const float* beta, void* out, int ldo, float* mean, float* rstd,
                         hipStream_t st) {
  if constexpr (sizeof(TI) == 4) {
    const int r = ln_rpw32();
    if (r == 1) return ln_fwd_launch_rpw<TI, 1>(out_dtype, rows, width, x, ldx, in_rows, gamma, beta, out, ldo, mean, rstd, st);
    if (r == 4) return ln_fwd_launch_rpw<TI, 4>(out_dtype, rows, width, x, ldx, in_rows, gamma, beta, out, ldo, mean, rstd, st);
  }
  return ln_fwd_launch_rpw<TI, CLIPK_LN_RPW>(out_dtype, rows, width, x, ldx, in_rows, gamma, beta, out, ldo, mean,
                                            rstd, st);
}

extern "C" int clipk_layernorm_fwd_x(int x_dtype, int out_dtype, int rows, int width, const void* x, int ldx,
                                     const int* in_rows, const float* gamma, const float* beta,
                                     void* out, int ldo, float* mean, float* rstd, void* stream) {
  if (!x || !gamma || !beta || !out) return CLIPK_EINVAL;
  if (rows < 0 || width <= 0 || width % 4 || width > 256 * LN_MAXV || ldx < width || ldo < width ||
      ldx % 4 || ldo % 4)
    return CLIPK_ESHAPE;
  if (rows == 0) return CLIPK_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (x_dtype) {
    case CLIPK_F32:
      return ln_fwd_launch<float>(out_dtype, rows, width, (const float*)x, ldx, in_rows, gamma, beta, out, ldo,
                                  mean, rstd, st);
    case CLIPK_F16:
      return ln_fwd_launch<f16>(out_dtype, rows, width, (const f16*)x, ldx, in_rows, gamma, beta, out, ldo, mean,
                                rstd, st);
    case CLIPK_BF16:
      return ln_fwd_launch<bf16>(out_dtype, rows, width, (const bf16*)x, ldx, in_rows, gamma, beta, out, ldo,
                                 mean, rstd, st);
    default: return CLIPK_EDTYPE;
  }
}

extern "C" int clipk_layernorm_fwd(int out_dtype, int rows, int width, const float* x, int ldx,
                                   const int* in_rows, const float* gamma, const float* beta,
                                   void* out, int ldo, float* mean, float* rstd, void* stream) {
  return clipk_layernorm_fwd_x(CLIPK_F32, out_dtype, rows, width, x, ldx, in_rows, gamma, beta, out, ldo, mean,
                               rstd, stream);
}

template <typename TD, typename TX>
static int ln_bwd_launch(int rows, int width, const void* dy, int lddy, const TX* x, int ldx,
                         const int* x_rows, const float* gamma, const float* mean, const float* rstd,
                         const void* dres, bool dres_lp, int lddres, float* dx, void* dx_lp, int lp_dtype,
                         const int* out_rows, int ldo, hipStream_t st) {
  constexpr int RPW = CLIPK_LN_RPW_BWD;
  dim3 grid((rows + 4 * RPW - 1) / (4 * RPW)), block(256);
  const TD* d = (const TD*)dy;
  const bool v8 = width % 512 == 0 && ldx % 8 == 0 && ldo % 8 == 0 && lddy % 8 == 0 && (!dres || lddres % 8 == 0);
  const bool one = v8 && width == 512;
#define CLIPK_LNB(TLP, RLV)                                                                                      \
  if (one)                                                                                                       \
    hipLaunchKernelGGL((ln_bwd_kernel<TLP, TD, TX, 8, RLV, 1, RPW>), grid, block, 0, st, rows, width, d, lddy, x, \
                       ldx, x_rows, gamma, mean, rstd, dres, lddres, dx, (TLP*)dx_lp, out_rows, ldo);            \
  else if (v8)                                                                                                   \
    hipLaunchKernelGGL((ln_bwd_kernel<TLP, TD, TX, 8, RLV, 2, RPW>), grid, block, 0, st, rows, width, d, lddy, x, \
                       ldx, x_rows, gamma, mean, rstd, dres, lddres, dx, (TLP*)dx_lp, out_rows, ldo);            \
  else                                                                                                           \
    hipLaunchKernelGGL((ln_bwd_kernel<TLP, TD, TX, 4, RLV, 4, RPW>), grid, block, 0, st, rows, width, d, lddy, x, \
                       ldx, x_rows, gamma, mean, rstd, dres, lddres, dx, (TLP*)dx_lp, out_rows, ldo);
  if (!dx_lp || lp_dtype == CLIPK_F32) {
    if (dres_lp) return CLIPK_EDTYPE;
    CLIPK_LNB(float, false)
  } else if (lp_dtype == CLIPK_F32S) {  // dx_lp: the next split GEMMs' pre-split A (fp32 gradients)
    if (dres_lp || ldo % 8) return CLIPK_EDTYPE;
    CLIPK_LNB(f32s, false)
  } else if (lp_dtype == CLIPK_BF16) {
    if (dres_lp) { CLIPK_LNB(bf16, true) } else { CLIPK_LNB(bf16, false) }
  } else if (lp_dtype == CLIPK_F16) {
    if (dres_lp) { CLIPK_LNB(f16, true) } else { CLIPK_LNB(f16, false) }
  } else {
    return CLIPK_EDTYPE;
  }
#undef CLIPK_LNB
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

template <typename TX>
static int ln_bwd_dy(int dy_dtype, int rows, int width, const void* dy, int lddy, const TX* x, int ldx,
                     const int* x_rows, const float* gamma, const float* mean, const float* rstd,
                     const void* dres, bool dres_lp, int lddres, float* dx, void* dx_lp, int lp_dtype,
                     const int* out_rows, int ldo, hipStream_t st) {
  switch (dy_dtype) {
    case CLIPK_F32:
      return ln_bwd_launch<float, TX>(rows, width, dy, lddy, x, ldx, x_rows, gamma, mean, rstd, dres, dres_lp,
                                      lddres, dx, dx_lp, lp_dtype, out_rows, ldo, st);
    case CLIPK_BF16:
      return ln_bwd_launch<bf16, TX>(rows, width, dy, lddy, x, ldx, x_rows, gamma, mean, rstd, dres, dres_lp,
                                     lddres, dx, dx_lp, lp_dtype, out_rows, ldo, st);
    case CLIPK_F16:
      return ln_bwd_launch<f16, TX>(rows, width, dy, lddy, x, ldx, x_rows, gamma, mean, rstd, dres, dres_lp,
                                    lddres, dx, dx_lp, lp_dtype, out_rows, ldo, st);
    default:
      return CLIPK_EDTYPE;
  }
}

extern "C" int clipk_layernorm_bwd_x2(int x_dtype, int dy_dtype, int rows, int width, const void* dy, int lddy,
                                      const void* x, int ldx, const int* x_rows, const float* gamma,
                                      const float* mean, const float* rstd, const void* dres, int dres_dtype,
                                      int lddres, float* dx, void* dx_lp, int lp_dtype,
                                      const int* out_rows, int ldo, void* stream) {
  const bool dres_lp = dres && dres_dtype != CLIPK_F32;
  if (dres_lp && (!dx_lp || dres_dtype != lp_dtype || lp_dtype == CLIPK_F32)) return CLIPK_EDTYPE;
  if (!dy || !x || !gamma || !mean || !rstd || (!dx && !dx_lp)) return CLIPK_EINVAL;
  if (rows < 0 || width <= 0 || width % 4 || width > 256 * LN_MAXV || ldx < width || ldo < width ||
      lddy < width || (dres && lddres < width))
    return CLIPK_ESHAPE;
  if (rows == 0) return CLIPK_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (x_dtype) {
    case CLIPK_F32:
      return ln_bwd_dy<float>(dy_dtype, rows, width, dy, lddy, (const float*)x, ldx, x_rows, gamma, mean, rstd,
                              dres, dres_lp, lddres, dx, dx_lp, lp_dtype, out_rows, ldo, st);
    case CLIPK_F16:
      return ln_bwd_dy<f16>(dy_dtype, rows, width, dy, lddy, (const f16*)x, ldx, x_rows, gamma, mean, rstd, dres,
                            dres_lp, lddres, dx, dx_lp, lp_dtype, out_rows, ldo, st);
    case CLIPK_BF16:
      return ln_bwd_dy<bf16>(dy_dtype, rows, width, dy, lddy, (const bf16*)x, ldx, x_rows, gamma, mean, rstd,
                             dres, dres_lp, lddres, dx, dx_lp, lp_dtype, out_rows, ldo, st);
    default:
      return CLIPK_EDTYPE;
  }
}

extern "C" int clipk_layernorm_bwd_x(int x_dtype, int dy_dtype, int rows, int width, const void* dy, int lddy,
                                     const void* x, int ldx, const int* x_rows, const float* gamma,
                                     const float* mean, const float* rstd, const float* dres,
                                     int lddres, float* dx, void* dx_lp, int lp_dtype,
                                     const int* out_rows, int ldo, void* stream) {
  if (!dx) return CLIPK_EINVAL;
  return clipk_layernorm_bwd_x2(x_dtype, dy_dtype, rows, width, dy, lddy, x, ldx, x_rows, gamma, mean, rstd, dres,
                                CLIPK_F32, lddres, dx, dx_lp, lp_dtype, out_rows, ldo, stream);
}

extern "C" int clipk_layernorm_bwd(int dy_dtype, int rows, int width, const void* dy, int lddy,
                                   const float* x, int ldx, const int* x_rows, const float* gamma,
                                   const float* mean, const float* rstd, const float* dres,
                                   int lddres, float* dx, void* dx_lp, int lp_dtype,
                                   const int* out_rows, int ldo, void* stream) {
  return clipk_layernorm_bwd_x(CLIPK_F32, dy_dtype, rows, width, dy, lddy, x, ldx, x_rows, gamma, mean, rstd,
                               dres, lddres, dx, dx_lp, lp_dtype, out_rows, ldo, stream);
}

namespace clipk {
// LayerNorm statistics from the per-(row, 64-column group) partials a clipk_gemm_ln producer
// wrote: (sum_g, M2_g = sum over the group of (x - sum_g / 64)^2). Exact merge (Chan et al.):
// mean = sum_g sum_g / width; M2 = sum_g M2_g + 64 (sum_g / 64 - mean)^2; rstd = 1 / sqrt(M2 /
// width + 1e-5) as model.py:153-159. Outputs (each optional): mean, rstd (the LayerNorm
// backward's), and rnb = (rstd, -rstd * mean) pairs (the folding GEMM's one 8-B load per row).
// LPR (8 or 16 >= width / 64) lanes per row, lane j holding partial j (8-B loads), sums over the
// LPR lanes by DPP in a fixed pattern (deterministic; idle lanes add exact zeros, so the 8- and
// 16-lane forms give the same bits). At >= 64k rows each lane group merges 4 rows whose loads are
// all issued before the first sum: one load per wave left the kernel latency-bound at 1.3 TB/s
// (26 us at the eval's 590k rows -> 13 us); below, one row per group keeps more blocks (the
// batch-1 step's 5.9k rows: 185 vs 47). The first form, one thread per row reading 64 B, took
// 5 us at 47k rows.
template <int CTRL>
__device__ __forceinline__ float dpp_row(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int LPR>
__device__ __forceinline__ float sum_lanes(float v) {
  v += dpp_row<0xB1>(v);   // quad: xor 1
  v += dpp_row<0x4E>(v);   // quad: xor 2
  v += dpp_row<0x141>(v);  // half-row mirror: quads 0 <-> 1
  if constexpr (LPR == 16) v += dpp_row<0x140>(v);  // row mirror: halves 0 <-> 1
  return v;
}
template <int LPR, int RPG>
__global__ __launch_bounds__(256) void ln_stats_merge_kernel(int rows, int ng, const f32x2* __restrict__ st,
                                                             float* __restrict__ mean, float* __restrict__ rstd,
                                                             f32x2* __restrict__ rnb) {
  constexpr int RPW = 64 / LPR;  // rows per wave and load
  const int lane = threadIdx.x & 63, j = lane % LPR;
  const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int r0 = wave * RPW * RPG + lane / LPR;
  f32x2 p[RPG];
#pragma unroll
  for (int k = 0; k < RPG; ++k) {
    const int r = r0 + k * RPW;
    p[k] = (r < rows && j < ng) ? st[(size_t)r * ng + j] : (f32x2){0.f, 0.f};
  }
  const float inv_w = 1.0f / (64.0f * ng);
#pragma unroll
  for (int k = 0; k < RPG; ++k) {
    const int r = r0 + k * RPW;
    const bool ok = r < rows && j < ng;
    const float mu = sum_lanes<LPR>(p[k][0]) * inv_w;
    const float d = p[k][0] * (1.0f / 64.0f) - mu;
    const float m2 = sum_lanes<LPR>(ok ? fmaf(64.0f * d, d, p[k][1]) : 0.f);
    if (r < rows && j == 0) {
      const float rs = rsqrtf(m2 * inv_w + 1e-5f);
      if (mean) mean[r] = mu;
      if (rstd) rstd[r] = rs;
      if (rnb) rnb[r] = (f32x2){rs, -rs * mu};
    }
  }
}
}  // namespace clipk

extern "C" int clipk_ln_stats_merge(int rows, int width, const float* stats, float* mean, float* rstd,
                                    float* rnb, void* stream) {
  if (!stats || (!mean && !rstd && !rnb)) return CLIPK_EINVAL;
  if (rows < 0 || width % 128 || width < 128 || width > 1024) return CLIPK_ESHAPE;
  if (rows == 0) return CLIPK_OK;
  const int ng = width / 64, lpr = ng <= 8 ? 8 : 16, rpg = rows >= 65536 ? 4 : 1;
  const long waves = ((long)rows + (64 / lpr) * rpg - 1) / ((64 / lpr) * rpg);
  const dim3 grid((unsigned)((waves + 3) / 4));
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, (hipStream_t)stream, rows, ng, reinterpret_cast<const f32x2*>(stats),
                       mean, rstd, reinterpret_cast<f32x2*>(rnb));
  };
  if (lpr == 8) {
    if (rpg == 4) go(ln_stats_merge_kernel<8, 4>);
    else go(ln_stats_merge_kernel<8, 1>);
  } else {
    if (rpg == 4) go(ln_stats_merge_kernel<16, 4>);
    else go(ln_stats_merge_kernel<16, 1>);
  }
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}
