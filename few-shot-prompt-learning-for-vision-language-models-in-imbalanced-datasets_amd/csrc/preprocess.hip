// Image preprocessing on the GPU: Pillow-exact bicubic resampling (two separable passes,
// 22-bit fixed-point coefficients, uint8 rounding + clipping after each pass) over a crop
// window, horizontal flip, and torchvision ToTensor + Normalize in fp32.
//
// Replaces the Dassl/torchvision PIL transforms (Dassl.pytorch/dassl/data/transforms/
// transforms.py:206-354: Resize + CenterCrop for test, RandomResizedCrop + flip for train)
// that run per image on the host. The coefficient tables (Pillow libImaging/Resample.c
// precompute_coeffs + normalize_coeffs_8bpc) are built on the host in float64
// (fsp_amd/data/preprocess.py); these kernels do the integer work. HBM/latency-bound: each
// output pixel reads ~ksize source pixels per pass.
#include "common.h"

namespace clipk {

constexpr int kPrecBits = 22;  // Pillow PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ int clip8(int s) {
  const int v = s >> kPrecBits;  // arithmetic shift, as Pillow's lookup index
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// desc (int64 x 16 per image): 0 src byte offset, 1 source row stride (pixels), 2 window
// left, 3 source row of temp row 0, 4 S, 5 flip, 6 h-table offset, 7 h ksize, 8 v-table
// offset, 9 v ksize, 10 temp byte offset, 11 temp rows, 12 source rows.
// h/v table rows: (first tap, taps used, ksize int32 coefficients).
__global__ __launch_bounds__(256) void resample_h_kernel(int B, int S, int rows_max, const uint8_t* __restrict__ src,
                                                         const long long* __restrict__ desc,
                                                         const int* __restrict__ tab, uint8_t* __restrict__ tmp) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long per = (long long)rows_max * S;
  if (i >= per * B) return;
  const int b = (int)(i / per);
  const int r = (int)((i % per) / S), x = (int)(i % S);
  const long long* d = desc + (size_t)b * 16;
  if (r >= (int)d[11]) return;
  const int ks = (int)d[7];
  const int* row = tab + d[6] + (size_t)x * (2 + ks);
  const int xmin = row[0], n = row[1];
  const uint8_t* p = src + d[0] + ((size_t)(d[3] + r) * d[1] + d[2] + xmin) * 3;
  int s0 = 1 << (kPrecBits - 1), s1 = s0, s2 = s0;
  for (int k = 0; k < n; ++k) {
    const int w = row[2 + k];
    s0 += (int)p[3 * k] * w;
    s1 += (int)p[3 * k + 1] * w;
    s2 += (int)p[3 * k + 2] * w;
  }
  uint8_t* o = tmp + d[10] + ((size_t)r * S + x) * 3;
  o[0] = (uint8_t)clip8(s0);
  o[1] = (uint8_t)clip8(s1);
  o[2] = (uint8_t)clip8(s2);
}

template <bool U8>
__global__ __launch_bounds__(256) void resample_v_kernel(int B, int S, const long long* __restrict__ desc,
                                                         const int* __restrict__ tab, const uint8_t* __restrict__ tmp,
                                                         const float* __restrict__ mean, const float* __restrict__ stdv,
                                                         void* __restrict__ out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long per = (long long)S * S;
  if (i >= per * B) return;
  const int b = (int)(i / per);
  const int y = (int)((i % per) / S), x = (int)(i % S);
  const long long* d = desc + (size_t)b * 16;
  const int ks = (int)d[9];
  const int* row = tab + d[8] + (size_t)y * (2 + ks);
  const int ymin = row[0], n = row[1];
  const uint8_t* t = tmp + d[10] + ((size_t)ymin * S + x) * 3;
  int s[3] = {1 << (kPrecBits - 1), 1 << (kPrecBits - 1), 1 << (kPrecBits - 1)};
  for (int k = 0; k < n; ++k) {
    const int w = row[2 + k];
#pragma unroll
    for (int c = 0; c < 3; ++c) s[c] += (int)t[(size_t)k * S * 3 + c] * w;
  }
  const int xo = d[5] ? S - 1 - x : x;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int v = clip8(s[c]);
    const size_t oi = (((size_t)b * 3 + c) * S + y) * S + xo;
    if constexpr (U8) {
      ((uint8_t*)out)[oi] = (uint8_t)v;
    } else {
      const float f = (float)v / 255.0f;          // ToTensor: float().div(255)
      ((float*)out)[oi] = (f - mean[c]) / stdv[c];  // Normalize: sub_(mean).div_(std)
    }
  }
}

}  // namespace clipk

using namespace clipk;

extern "C" int clipk_image_resample(int B, int S, int rows_max, const void* src, const long long* desc,
                                    const int* tables, void* tmp, const float* mean, const float* stdv,
                                    int out_uint8, void* out, void* stream) {
  if (!src || !desc || !tables || !tmp || !out || (!out_uint8 && (!mean || !stdv))) return CLIPK_EINVAL;
  if (B < 0 || S <= 0 || rows_max <= 0) return CLIPK_ESHAPE;
  if (B == 0) return CLIPK_OK;
  hipStream_t st = (hipStream_t)stream;
  const long long nh = (long long)B * rows_max * S, nv = (long long)B * S * S;
  hipLaunchKernelGGL(resample_h_kernel, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, st, B, S, rows_max,
                     (const uint8_t*)src, desc, tables, (uint8_t*)tmp);
  CLIPK_CHECK_LAUNCH();
  if (out_uint8)
    hipLaunchKernelGGL(resample_v_kernel<true>, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, B, S, desc,
                       tables, (const uint8_t*)tmp, mean, stdv, out);
  else
    hipLaunchKernelGGL(resample_v_kernel<false>, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, B, S, desc,
                       tables, (const uint8_t*)tmp, mean, stdv, out);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}
