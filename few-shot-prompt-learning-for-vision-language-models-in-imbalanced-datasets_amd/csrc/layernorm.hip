// LayerNorm forward / input-grad backward as wavefront row reductions (HBM-bound).
// Reference: PromptSRC/clip/model.py:153-159 (fp32 upcast, eps 1e-5, affine).
// One wave per row, the row kept in registers (width <= 1024), two-pass mean/variance from
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
  if constexpr (VW == 4) {
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

template <typename TI, typename TO, int VW>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int rows, int width, const TI* __restrict__ x,
                                                     int ldx, const int* __restrict__ in_rows,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, TO* __restrict__ out,
                                                     int ldo, float* __restrict__ mean,
                                                     float* __restrict__ rstd) {
  constexpr int NC = 1024 / (64 * VW);
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int xr = in_rows ? in_rows[r] : r;
  const TI* xp = x + (size_t)xr * ldx;
  const int nv = width / VW;  // vectors per row
  float v[NC][VW], gg[NC][VW], bb[NC][VW];
  float s = 0.f;
  // gamma / beta are issued with x: loaded after the two reductions they were one more
  // dependent round trip per row
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + i * 64;
    if (c < nv) {
      ldv<TI, VW>(xp + c * VW, v[i]);
      ldv<float, VW>(gamma + c * VW, gg[i]);
      ldv<float, VW>(beta + c * VW, bb[i]);
#pragma unroll
      for (int k = 0; k < VW; ++k) s += v[i][k];
    } else {
#pragma unroll
      for (int k = 0; k < VW; ++k) v[i][k] = 0.f;
    }
  }
  const float inv_w = 1.0f / (float)width;
  const float mu = wave_sum(s) * inv_w;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + i * 64;
    if (c < nv) {
#pragma unroll
      for (int k = 0; k < VW; ++k) { const float d = v[i][k] - mu; q += d * d; }
    }
  }
  const float rs = rsqrtf(wave_sum(q) * inv_w + 1e-5f);
  TO* op = out + (size_t)r * ldo;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + i * 64;
    if (c < nv) {
      float o[VW];
#pragma unroll
      for (int k = 0; k < VW; ++k) o[k] = (v[i][k] - mu) * rs * gg[i][k] + bb[i][k];
      stv<TO, VW>(op + c * VW, o);
    }
  }
  if (lane == 0) {
    if (mean) mean[r] = mu;
    if (rstd) rstd[r] = rs;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) + dres,   g = dy * gamma
// RL: the incoming residual gradient dres is in the low-precision dtype TL (a 16-bit residual-
// gradient stream, updated in place: dres == dx_lp is allowed, each lane reads its chunk
// before writing it); dx (fp32) may then be null.
template <typename TL, typename TD, typename TX, int VW, bool RL = false>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int rows, int width, const TD* __restrict__ dy,
                                                     int lddy, const TX* __restrict__ x, int ldx,
                                                     const int* __restrict__ x_rows,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd,
                                                     const void* dres_v, int lddres,
                                                     float* __restrict__ dx, TL* dx_lp,
                                                     const int* __restrict__ out_rows, int ldo) {
  constexpr int NC = 1024 / (64 * VW);
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int xr = x_rows ? x_rows[r] : r;
  const int orow = out_rows ? out_rows[r] : r;
  const float mu = mean[r], rs = rstd[r];
  const TX* xp = x + (size_t)xr * ldx;
  const TD* dp = dy + (size_t)r * lddy;
  const int nv = width / VW;
  float gv[NC][VW], xh[NC][VW], rv[NC][VW];
  float s1 = 0.f, s2 = 0.f;
  typedef typename std::conditional<RL, TL, float>::type TR;
  const TR* rp = dres_v ? (const TR*)dres_v + (size_t)orow * lddres : nullptr;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + i * 64;
    if (c < nv) {
      float xv[VW], dv[VW], gg[VW];
      ldv<TX, VW>(xp + c * VW, xv);
      ldv<TD, VW>(dp + c * VW, dv);
      ldv<float, VW>(gamma + c * VW, gg);
      // the residual gradient is issued with the other operands (not after the reductions)
      if (rp) ldv<TR, VW>(rp + c * VW, rv[i]);
#pragma unroll
      for (int k = 0; k < VW; ++k) {
        xh[i][k] = (xv[k] - mu) * rs;
        gv[i][k] = dv[k] * gg[k];
        s1 += gv[i][k];
        s2 += gv[i][k] * xh[i][k];
      }
    }
  }
  const float inv_w = 1.0f / (float)width;
  const float m1 = wave_sum(s1) * inv_w;
  const float m2 = wave_sum(s2) * inv_w;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + i * 64;
    if (c < nv) {
      float o[VW];
#pragma unroll
      for (int k = 0; k < VW; ++k) o[k] = rs * (gv[i][k] - m1 - xh[i][k] * m2);
      if (rp) {
#pragma unroll
        for (int k = 0; k < VW; ++k) o[k] += rv[i][k];
      }
      if (dx) stv<float, VW>(dx + (size_t)orow * ldo + c * VW, o);
      if (dx_lp) stv<TL, VW>(dx_lp + (size_t)orow * ldo + c * VW, o);
    }
  }
}

}  // namespace clipk

using namespace clipk;

template <typename TI>
static int ln_fwd_launch(int out_dtype, int rows, int width, const TI* x, int ldx, const int* in_rows,
                         const float* gamma, const float* beta, void* out, int ldo, float* mean, float* rstd,
                         hipStream_t st) {
  dim3 grid((rows + 3) / 4), block(256);
  const bool v8 = width % 512 == 0 && ldx % 8 == 0 && ldo % 8 == 0;
#define CLIPK_LNF(TOUT)                                                                                       \
  if (v8)                                                                                                     \
    hipLaunchKernelGGL((ln_fwd_kernel<TI, TOUT, 8>), grid, block, 0, st, rows, width, x, ldx, in_rows, gamma, \
                       beta, (TOUT*)out, ldo, mean, rstd);                                                    \
  else                                                                                                        \
    hipLaunchKernelGGL((ln_fwd_kernel<TI, TOUT, 4>), grid, block, 0, st, rows, width, x, ldx, in_rows, gamma, \
                       beta, (TOUT*)out, ldo, mean, rstd);
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
  dim3 grid((rows + 3) / 4), block(256);
  const TD* d = (const TD*)dy;
  const bool v8 = width % 512 == 0 && ldx % 8 == 0 && ldo % 8 == 0 && lddy % 8 == 0 && (!dres || lddres % 8 == 0);
#define CLIPK_LNB(TLP, RLV)                                                                                     \
  if (v8)                                                                                                       \
    hipLaunchKernelGGL((ln_bwd_kernel<TLP, TD, TX, 8, RLV>), grid, block, 0, st, rows, width, d, lddy, x, ldx,   \
                       x_rows, gamma, mean, rstd, dres, lddres, dx, (TLP*)dx_lp, out_rows, ldo);                \
  else                                                                                                          \
    hipLaunchKernelGGL((ln_bwd_kernel<TLP, TD, TX, 4, RLV>), grid, block, 0, st, rows, width, d, lddy, x, ldx,   \
                       x_rows, gamma, mean, rstd, dres, lddres, dx, (TLP*)dx_lp, out_rows, ldo);
  if (!dx_lp || lp_dtype == CLIPK_F32) {
    if (dres_lp) return CLIPK_EDTYPE;
    CLIPK_LNB(float, false)
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
