// Is v_mfma_f32_16x16x32_f16 with all-zero products an identity on C? (lab, not in libclipk.so)
// Each of 64 lanes x 4 accumulators holds random fp32 C values over a wide exponent range;
// D = mfma(B = 0, A = random f16, C), then the same with A = 0, then D = C + 0 products from a
// second MFMA whose products are exact small values. Prints how many D != C.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const float* c_in, const _Float16* a_in, float* d0, float* d1, int n) {
  const int lane = threadIdx.x & 63;
  const int blk = blockIdx.x;
  if (blk * 256 >= n) return;
  f32x4 c;
  for (int r = 0; r < 4; ++r) c[r] = c_in[blk * 256 + lane * 4 + r];
  f16x8 a, z;
  for (int e = 0; e < 8; ++e) { a[e] = a_in[(blk * 64 + lane) * 8 + e]; z[e] = (_Float16)0.0f; }
  f32x4 x = __builtin_amdgcn_mfma_f32_16x16x32_f16(z, a, c, 0, 0, 0);
  f32x4 y = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, z, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) { d0[blk * 256 + lane * 4 + r] = x[r]; d1[blk * 256 + lane * 4 + r] = y[r]; }
}

int main() {
  const int nb = 4096, n = nb * 256;
  float* c = (float*)malloc(n * 4); _Float16* a = (_Float16*)malloc(n * 2 * 2);
  srand(1);
  for (int i = 0; i < n; ++i) {
    float u = (rand() / (float)RAND_MAX) * 2 - 1;
    c[i] = u * ldexpf(1.0f, rand() % 40 - 20);
  }
  for (int i = 0; i < 2 * n; ++i) a[i] = (_Float16)((rand() / (float)RAND_MAX) * 2 - 1);
  float *dc, *d0, *d1; _Float16* da;
  hipMalloc(&dc, n * 4); hipMalloc(&d0, n * 4); hipMalloc(&d1, n * 4); hipMalloc(&da, n * 4);
  hipMemcpy(dc, c, n * 4, hipMemcpyHostToDevice); hipMemcpy(da, a, n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(nb), dim3(64), 0, 0, dc, da, d0, d1, n);
  float* h0 = (float*)malloc(n * 4); float* h1 = (float*)malloc(n * 4);
  hipMemcpy(h0, d0, n * 4, hipMemcpyDeviceToHost); hipMemcpy(h1, d1, n * 4, hipMemcpyDeviceToHost);
  long bad0 = 0, bad1 = 0; double worst = 0;
  for (int i = 0; i < n; ++i) {
    if (memcmp(&h0[i], &c[i], 4)) { ++bad0; worst = fmax(worst, fabs((h0[i] - c[i]) / c[i])); if (bad0 <= 5) printf("C %.9g -> %.9g\n", c[i], h0[i]); }
    if (memcmp(&h1[i], &c[i], 4)) ++bad1;
  }
  printf("zero B: %ld of %d changed (worst rel %.3g); zero A: %ld changed\n", bad0, n / 4 * 0 + n, worst, bad1);
  return 0;
}
