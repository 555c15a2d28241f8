// LayerNorm forward / input-grad backward as wavefront row reductions (HBM-bound).
// Reference: PromptSRC/clip/model.py:153-159 (fp32 upcast, eps 1e-5, affine).
// One wave per row, 4-element vector loads, the row kept in registers (width <= 1024 ->
// <= 4 vectors per lane), two-pass mean/variance from registers (no E[x^2]-E[x]^2
// cancellation). The input row (the residual stream) is fp32 or, for the 16-bit text
// residual stream, the activation dtype (statistics always in fp32). Optional row gather (in_rows) for ln_final on EOT rows and ln_post on
// CLS rows, optional scatter (out_rows) on the backward.
#include "common.h"

namespace clipk {

constexpr int LN_MAXV = 4;  // float4 per lane -> width <= 1024

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int rows, int width, const TI* __restrict__ x,
                                                     int ldx, const int* __restrict__ in_rows,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, TO* __restrict__ out,
                                                     int ldo, float* __restrict__ mean,
                                                     float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int xr = in_rows ? in_rows[r] : r;
  const TI* xp = x + (size_t)xr * ldx;
  const int nv = width >> 2;  // 4-element vector count
  f32x4 v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + i * 64;
    if (c < nv) {
      float t4[4];
      load4<TI>(xp + c * 4, t4);
      v[i] = (f32x4){t4[0], t4[1], t4[2], t4[3]};
      s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
    } else {
      v[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  }
  const float inv_w = 1.0f / (float)width;
  const float mu = wave_sum(s) * inv_w;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + i * 64;
    if (c < nv) {
#pragma unroll
      for (int k = 0; k < 4; ++k) { const float d = v[i][k] - mu; q += d * d; }
    }
  }
  const float rs = rsqrtf(wave_sum(q) * inv_w + 1e-5f);
  TO* op = out + (size_t)r * ldo;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + i * 64;
    if (c < nv) {
      const f32x4 gg = reinterpret_cast<const f32x4*>(gamma)[c];
      const f32x4 bb = reinterpret_cast<const f32x4*>(beta)[c];
      store4<TO>(op + c * 4, (v[i][0] - mu) * rs * gg[0] + bb[0], (v[i][1] - mu) * rs * gg[1] + bb[1],
                 (v[i][2] - mu) * rs * gg[2] + bb[2], (v[i][3] - mu) * rs * gg[3] + bb[3]);
    }
  }
  if (lane == 0) {
    if (mean) mean[r] = mu;
    if (rstd) rstd[r] = rs;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) + dres,   g = dy * gamma
template <typename TL, typename TD, typename TX>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int rows, int width, const TD* __restrict__ dy,
                                                     int lddy, const TX* __restrict__ x, int ldx,
                                                     const int* __restrict__ x_rows,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd,
                                                     const float* __restrict__ dres, int lddres,
                                                     float* __restrict__ dx, TL* __restrict__ dx_lp,
                                                     const int* __restrict__ out_rows, int ldo) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int xr = x_rows ? x_rows[r] : r;
  const int orow = out_rows ? out_rows[r] : r;
  const float mu = mean[r], rs = rstd[r];
  const TX* xp = x + (size_t)xr * ldx;
  const TD* dp = dy + (size_t)r * lddy;
  const int nv = width >> 2;
  f32x4 gv[LN_MAXV], xh[LN_MAXV];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + i * 64;
    if (c < nv) {
      float xva[4];
      load4<TX>(xp + c * 4, xva);
      const f32x4 xv = {xva[0], xva[1], xva[2], xva[3]};
      float dva[4];
      load4<TD>(dp + c * 4, dva);
      const f32x4 dv = {dva[0], dva[1], dva[2], dva[3]};
      const f32x4 gg = reinterpret_cast<const f32x4*>(gamma)[c];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
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
  float* op = dx + (size_t)orow * ldo;
  const float* rp = dres ? dres + (size_t)orow * lddres : nullptr;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + i * 64;
    if (c < nv) {
      f32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = rs * (gv[i][k] - m1 - xh[i][k] * m2);
      if (rp) {
        const f32x4 rv = reinterpret_cast<const f32x4*>(rp)[c];
        o += rv;
      }
      reinterpret_cast<f32x4*>(op)[c] = o;
      if (dx_lp) store4<TL>(dx_lp + (size_t)orow * ldo + c * 4, o[0], o[1], o[2], o[3]);
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
  switch (out_dtype) {
    case CLIPK_F32:
      hipLaunchKernelGGL((ln_fwd_kernel<TI, float>), grid, block, 0, st, rows, width, x, ldx, in_rows, gamma, beta,
                         (float*)out, ldo, mean, rstd);
      break;
    case CLIPK_F16:
      hipLaunchKernelGGL((ln_fwd_kernel<TI, f16>), grid, block, 0, st, rows, width, x, ldx, in_rows, gamma, beta,
                         (f16*)out, ldo, mean, rstd);
      break;
    case CLIPK_BF16:
      hipLaunchKernelGGL((ln_fwd_kernel<TI, bf16>), grid, block, 0, st, rows, width, x, ldx, in_rows, gamma, beta,
                         (bf16*)out, ldo, mean, rstd);
      break;
    default: return CLIPK_EDTYPE;
  }
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
                         const float* dres, int lddres, float* dx, void* dx_lp, int lp_dtype,
                         const int* out_rows, int ldo, hipStream_t st) {
  dim3 grid((rows + 3) / 4), block(256);
  const TD* d = (const TD*)dy;
  if (!dx_lp || lp_dtype == CLIPK_F32) {
    hipLaunchKernelGGL((ln_bwd_kernel<float, TD, TX>), grid, block, 0, st, rows, width, d, lddy, x, ldx,
                       x_rows, gamma, mean, rstd, dres, lddres, dx, (float*)dx_lp, out_rows, ldo);
  } else if (lp_dtype == CLIPK_BF16) {
    hipLaunchKernelGGL((ln_bwd_kernel<bf16, TD, TX>), grid, block, 0, st, rows, width, d, lddy, x, ldx,
                       x_rows, gamma, mean, rstd, dres, lddres, dx, (bf16*)dx_lp, out_rows, ldo);
  } else if (lp_dtype == CLIPK_F16) {
    hipLaunchKernelGGL((ln_bwd_kernel<f16, TD, TX>), grid, block, 0, st, rows, width, d, lddy, x, ldx,
                       x_rows, gamma, mean, rstd, dres, lddres, dx, (f16*)dx_lp, out_rows, ldo);
  } else {
    return CLIPK_EDTYPE;
  }
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

template <typename TX>
static int ln_bwd_dy(int dy_dtype, int rows, int width, const void* dy, int lddy, const TX* x, int ldx,
                     const int* x_rows, const float* gamma, const float* mean, const float* rstd,
                     const float* dres, int lddres, float* dx, void* dx_lp, int lp_dtype,
                     const int* out_rows, int ldo, hipStream_t st) {
  switch (dy_dtype) {
    case CLIPK_F32:
      return ln_bwd_launch<float, TX>(rows, width, dy, lddy, x, ldx, x_rows, gamma, mean, rstd, dres, lddres,
                                      dx, dx_lp, lp_dtype, out_rows, ldo, st);
    case CLIPK_BF16:
      return ln_bwd_launch<bf16, TX>(rows, width, dy, lddy, x, ldx, x_rows, gamma, mean, rstd, dres, lddres,
                                     dx, dx_lp, lp_dtype, out_rows, ldo, st);
    case CLIPK_F16:
      return ln_bwd_launch<f16, TX>(rows, width, dy, lddy, x, ldx, x_rows, gamma, mean, rstd, dres, lddres,
                                    dx, dx_lp, lp_dtype, out_rows, ldo, st);
    default:
      return CLIPK_EDTYPE;
  }
}

extern "C" int clipk_layernorm_bwd_x(int x_dtype, int dy_dtype, int rows, int width, const void* dy, int lddy,
                                     const void* x, int ldx, const int* x_rows, const float* gamma,
                                     const float* mean, const float* rstd, const float* dres,
                                     int lddres, float* dx, void* dx_lp, int lp_dtype,
                                     const int* out_rows, int ldo, void* stream) {
  if (!dy || !x || !gamma || !mean || !rstd || !dx) return CLIPK_EINVAL;
  if (rows < 0 || width <= 0 || width % 4 || width > 256 * LN_MAXV || ldx < width || ldo < width ||
      lddy < width || (dres && lddres < width))
    return CLIPK_ESHAPE;
  if (rows == 0) return CLIPK_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (x_dtype) {
    case CLIPK_F32:
      return ln_bwd_dy<float>(dy_dtype, rows, width, dy, lddy, (const float*)x, ldx, x_rows, gamma, mean, rstd,
                              dres, lddres, dx, dx_lp, lp_dtype, out_rows, ldo, st);
    case CLIPK_F16:
      return ln_bwd_dy<f16>(dy_dtype, rows, width, dy, lddy, (const f16*)x, ldx, x_rows, gamma, mean, rstd, dres,
                            lddres, dx, dx_lp, lp_dtype, out_rows, ldo, st);
    case CLIPK_BF16:
      return ln_bwd_dy<bf16>(dy_dtype, rows, width, dy, lddy, (const bf16*)x, ldx, x_rows, gamma, mean, rstd,
                             dres, lddres, dx, dx_lp, lp_dtype, out_rows, ldo, st);
    default:
      return CLIPK_EDTYPE;
  }
}

extern "C" int clipk_layernorm_bwd(int dy_dtype, int rows, int width, const void* dy, int lddy,
                                   const float* x, int ldx, const int* x_rows, const float* gamma,
                                   const float* mean, const float* rstd, const float* dres,
                                   int lddres, float* dx, void* dx_lp, int lp_dtype,
                                   const int* out_rows, int ldo, void* stream) {
  return clipk_layernorm_bwd_x(CLIPK_F32, dy_dtype, rows, width, dy, lddy, x, ldx, x_rows, gamma, mean, rstd,
                               dres, lddres, dx, dx_lp, lp_dtype, out_rows, ldo, stream);
}
