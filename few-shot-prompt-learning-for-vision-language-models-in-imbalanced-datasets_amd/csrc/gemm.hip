// MFMA GEMM with fused epilogues for every linear layer on the CoOp/CoCoOp path:
//   out[M,N] = epilogue( A[M,K] . B[N,K]^T ),  fp32 accumulate.
// A = activations (row-major, K contiguous), B = packed frozen weight (row-major [N,K]),
// i.e. the nn.Linear layout (PromptSRC/clip/model.py:171-177) and its transpose for
// the input-grad GEMMs (pre-packed once, so backward is the same "NT" form).
//
// gfx950 design:
//  * 256 threads = 4 waves (2x2), block tile 128x128, K staged 128 bytes per row
//    (64 halfs or 32 floats) into a 2-stage LDS ring by global_load_lds_dwordx4 (glds):
//    one wave-instruction = 8 rows x 128 B = 1 KiB, lane-linear in LDS.
//  * LDS image row-swizzled on the SOURCE address (glds writes lane-linear): physical
//    16-B chunk p = c ^ ((row >> 1) & 7). With rows = lane&15 read by ds_read_b128 this
//    puts each 16-lane group on 16 distinct 16-B slots of the 256-B bank row (no conflict).
//  * MFMA v_mfma_f32_16x16x32_{f16,bf16} (or v_mfma_f32_16x16x4_f32 for the fp32 parity
//    mode) with SWAPPED operands (weights as the A operand): each lane then holds 4
//    consecutive output columns of one row, so the epilogue issues 8/16-B row stores and
//    float4 bias/residual loads.
//  * XCD-aware bijective block remap: consecutive tiles of one A row-panel run on one XCD
//    so the panel is fetched from HBM once and re-read from that XCD's L2.
#include "common.h"

namespace clipk {

constexpr int GEMM_BM = 128;
constexpr int GEMM_BN = 128;
constexpr int GEMM_ROWB = 128;                         // bytes per staged row (BK)
constexpr int GEMM_OPB = GEMM_BM * GEMM_ROWB;          // 16 KiB per operand per stage
constexpr int GEMM_STAGEB = 2 * GEMM_OPB;              // A + B
constexpr int GEMM_LDS = 2 * GEMM_STAGEB;              // 2 stages = 64 KiB

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct GemmArgs {
  const char* A; const char* B;
  int M, N, K, lda, ldb;            // lda/ldb in elements
  const float* bias; const float* res; int ldr;
  void* out; int ldo; void* out2;
  const void* aux; int ldaux;
};

template <typename T>
__device__ __forceinline__ f32x4 mma(u32x4 a, u32x4 b, f32x4 c) {
  if constexpr (sizeof(T) == 4) {
    f32x4 fa = __builtin_bit_cast(f32x4, a);
    f32x4 fb = __builtin_bit_cast(f32x4, b);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[0], fb[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[1], fb[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[2], fb[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[3], fb[3], c, 0, 0, 0);
    return c;
  } else if constexpr (__is_same(T, f16)) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
}

__device__ __forceinline__ void glds16(const char* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(
      (const __attribute__((address_space(1))) void*)src,
      (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

template <typename T, typename TO, typename TX, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(GemmArgs g) {
  __shared__ CLIPK_LDS_ALIGN char smem[GEMM_LDS];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // ---- XCD-aware bijective tile remap (tiles of one A row-panel share an XCD).
  const int ntn = g.N / GEMM_BN;
  const int ntm = (g.M + GEMM_BM - 1) / GEMM_BM;
  const int nwg = ntm * ntn;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int m0 = (wgid / ntn) * GEMM_BM;
  const int n0 = (wgid % ntn) * GEMM_BN;

  // ---- staging addresses: this wave stages rows [w*32, w*32+32) of A and of B.
  const size_t esz = sizeof(T);
  const char* srcA[4];
  const char* srcB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = w * 32 + i * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    int ga = m0 + row;
    ga = ga < g.M ? ga : g.M - 1;
    srcA[i] = g.A + ((size_t)ga * g.lda) * esz + c * 16;
    srcB[i] = g.B + ((size_t)(n0 + row) * g.ldb) * esz + c * 16;
  }
  auto stage = [&](int s, int kt) {
    char* base = smem + s * GEMM_STAGEB;
    const size_t koff = (size_t)kt * GEMM_ROWB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      glds16(srcA[i] + koff, base + (w * 32 + i * 8) * GEMM_ROWB);
      glds16(srcB[i] + koff, base + GEMM_OPB + (w * 32 + i * 8) * GEMM_ROWB);
    }
  };

  const int wm = w >> 1, wn = w & 1;
  const int fr = lane & 15;         // fragment row within a 16-row sub-tile
  const int fq = lane >> 4;         // 16-B chunk within a 64-B k-window
  const int sw = (fr >> 1) & 7;     // row swizzle (row base is a multiple of 16)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (int)((size_t)g.K * esz / GEMM_ROWB);
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
    const char* As = smem + cur * GEMM_STAGEB + (wm * 64 + fr) * GEMM_ROWB;
    const char* Bs = smem + cur * GEMM_STAGEB + GEMM_OPB + (wn * 64 + fr) * GEMM_ROWB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int p = ((kk * 4 + fq) ^ sw) * 16;
      u32x4 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const u32x4*>(As + i * 16 * GEMM_ROWB + p);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const u32x4*>(Bs + j * 16 * GEMM_ROWB + p);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mma<T>(b[j], a[i], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: lane holds C[m][n..n+3]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + fr;
    if (m >= g.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + fq * 4;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if constexpr (EPI == CLIPK_EPI_BIAS || EPI == CLIPK_EPI_BIAS_RES || EPI == CLIPK_EPI_BIAS_QGELU) {
        f32x4 bb = *reinterpret_cast<const f32x4*>(g.bias + n);
        v[0] += bb[0]; v[1] += bb[1]; v[2] += bb[2]; v[3] += bb[3];
      }
      if constexpr (EPI == CLIPK_EPI_BIAS_RES) {
        const f32x4 rr = *reinterpret_cast<const f32x4*>(g.res + (size_t)m * g.ldr + n);
        f32x4 o = {v[0] + rr[0], v[1] + rr[1], v[2] + rr[2], v[3] + rr[3]};
        *reinterpret_cast<f32x4*>((float*)g.out + (size_t)m * g.ldo + n) = o;
      } else if constexpr (EPI == CLIPK_EPI_BIAS_QGELU) {
        if (g.out2) store4<TO>((TO*)g.out2 + (size_t)m * g.ldo + n, v[0], v[1], v[2], v[3]);
        store4<TO>((TO*)g.out + (size_t)m * g.ldo + n, quick_gelu(v[0]), quick_gelu(v[1]),
                   quick_gelu(v[2]), quick_gelu(v[3]));
      } else if constexpr (EPI == CLIPK_EPI_DQGELU) {
        float h[4];
        load4<TX>((const TX*)g.aux + (size_t)m * g.ldaux + n, h);
        store4<TO>((TO*)g.out + (size_t)m * g.ldo + n, v[0] * quick_gelu_grad(h[0]),
                   v[1] * quick_gelu_grad(h[1]), v[2] * quick_gelu_grad(h[2]),
                   v[3] * quick_gelu_grad(h[3]));
      } else {
        store4<TO>((TO*)g.out + (size_t)m * g.ldo + n, v[0], v[1], v[2], v[3]);
      }
    }
  }
}

template <typename T, typename TO, typename TX, int EPI>
static int launch_gemm(const GemmArgs& g, hipStream_t st) {
  const int nwg = ((g.M + GEMM_BM - 1) / GEMM_BM) * (g.N / GEMM_BN);
  hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI>), dim3(nwg), dim3(256), 0, st, g);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

// dtype dispatch: (in, out, epi[, aux])
template <typename T>
static int dispatch_out(int out_dtype, int epi, int aux_dtype, const GemmArgs& g, hipStream_t st) {
  if (epi == CLIPK_EPI_BIAS_RES) {
    if (out_dtype != CLIPK_F32) return CLIPK_EDTYPE;
    return launch_gemm<T, float, float, CLIPK_EPI_BIAS_RES>(g, st);
  }
  if (epi == CLIPK_EPI_DQGELU) {
    // backward: out in the grad dtype (== T), aux = forward pre-activation
    if (out_dtype != DT<T>::id) return CLIPK_EDTYPE;
    if (aux_dtype == CLIPK_F16) return launch_gemm<T, T, f16, CLIPK_EPI_DQGELU>(g, st);
    if (aux_dtype == CLIPK_BF16) return launch_gemm<T, T, bf16, CLIPK_EPI_DQGELU>(g, st);
    if (aux_dtype == CLIPK_F32) return launch_gemm<T, T, float, CLIPK_EPI_DQGELU>(g, st);
    return CLIPK_EDTYPE;
  }
#define CLIPK_OUTS(EPIV)                                                           \
  switch (out_dtype) {                                                             \
    case CLIPK_F32: return launch_gemm<T, float, float, EPIV>(g, st);              \
    case CLIPK_F16: return launch_gemm<T, f16, float, EPIV>(g, st);                \
    case CLIPK_BF16: return launch_gemm<T, bf16, float, EPIV>(g, st);              \
    default: return CLIPK_EDTYPE;                                                  \
  }
  if (epi == CLIPK_EPI_BIAS) { CLIPK_OUTS(CLIPK_EPI_BIAS) }
  if (epi == CLIPK_EPI_BIAS_QGELU) {
    if (out_dtype == CLIPK_F32 && sizeof(T) != 4) return CLIPK_EDTYPE;
    CLIPK_OUTS(CLIPK_EPI_BIAS_QGELU)
  }
  if (epi == CLIPK_EPI_NONE) { CLIPK_OUTS(CLIPK_EPI_NONE) }
#undef CLIPK_OUTS
  return CLIPK_EINVAL;
}

}  // namespace clipk

using namespace clipk;

extern "C" int clipk_gemm(int in_dtype, int out_dtype, int epi, int M, int N, int K,
                          const void* A, int lda, const void* B, int ldb,
                          const float* bias, const float* res, int ldr,
                          void* out, int ldo, void* out2, const void* aux, int aux_dtype,
                          int ldaux, void* stream) {
  if (!A || !B || !out) return CLIPK_EINVAL;
  if (M <= 0) return M == 0 ? CLIPK_OK : CLIPK_ESHAPE;
  const int esz = in_dtype == CLIPK_F32 ? 4 : 2;
  if (N <= 0 || K <= 0 || N % GEMM_BN != 0 || (K * esz) % GEMM_ROWB != 0) return CLIPK_ESHAPE;
  if (lda < K || ldb < K || (lda * esz) % 16 || (ldb * esz) % 16 || ldo < N || ldo % 4)
    return CLIPK_ESHAPE;
  if ((epi == CLIPK_EPI_BIAS || epi == CLIPK_EPI_BIAS_RES || epi == CLIPK_EPI_BIAS_QGELU) && !bias)
    return CLIPK_EINVAL;
  if (epi == CLIPK_EPI_BIAS_RES && (!res || ldr < N || ldr % 4)) return CLIPK_EINVAL;
  if (epi == CLIPK_EPI_DQGELU && (!aux || ldaux < N || ldaux % 4)) return CLIPK_EINVAL;
  GemmArgs g{(const char*)A, (const char*)B, M, N, K, lda, ldb, bias, res, ldr, out, ldo, out2, aux,
             ldaux};
  hipStream_t st = (hipStream_t)stream;
  switch (in_dtype) {
    case CLIPK_F16: return dispatch_out<f16>(out_dtype, epi, aux_dtype, g, st);
    case CLIPK_BF16: return dispatch_out<bf16>(out_dtype, epi, aux_dtype, g, st);
    case CLIPK_F32: return dispatch_out<float>(out_dtype, epi, aux_dtype, g, st);
    default: return CLIPK_EDTYPE;
  }
}
