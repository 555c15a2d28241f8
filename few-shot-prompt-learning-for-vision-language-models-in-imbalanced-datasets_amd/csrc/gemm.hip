// libclipk GEMM entry points (include/clipk.h): clipk_gemm, the LayerNorm-fold forms, split-K, the
// PREC fp32s weight packing. The kernel template lives in gemm_kernel.h.
#include "gemm_kernel.h"

namespace clipk {

// the kernel's SPF bits from the C-ABI's operand flags (include/clipk.h)
static int split_flags(int epi) {
  return ((epi & CLIPK_A_SPLIT) ? 1 : 0) | ((epi & CLIPK_OUT_SPLIT) ? 2 : 0) | ((epi & CLIPK_OUT2_SPLIT_GAMMA) ? 4 : 0);
}

// Tile configurations: 0 = 128x128 (4 waves, 64 KiB LDS, 2 blocks/CU),
// 1 = 256x256 (8 waves, 128 KiB, persistent when the grid exceeds 2 waves of CUs),
// 2 = 256x128 (8 waves, 96 KiB), 3 = 256x256 non-persistent (benchmark knob),
// 6 = 192x256 (8 waves of 96x64, 112 KiB + scratch): 4/3 more row tiles, chosen when it
// fills the last wave of CUs better than 256-row tiles (N = 512 at 47k rows: 1.45 -> 1.92
// waves).
static int g_force_cfg = -2;  // -2: unread, -1: auto
int pick_cfg(int M, int N, int esz) {
  if (g_force_cfg == -2) {
    const char* e = getenv("CLIPK_GEMM_CFG");
    g_force_cfg = e ? atoi(e) : -1;
  }
  if (esz == 4) return 0;  // fp32 parity path: one configuration
  if (g_force_cfg >= 0) {
    if ((g_force_cfg == 1 || g_force_cfg == 3 || g_force_cfg == 6) && N % 256 == 0) return g_force_cfg;
    if (g_force_cfg == 7) return g_force_cfg;
    if (g_force_cfg == 2) return g_force_cfg;
    return 0;
  }
  // small M (the ViT at training batch sizes): 64x128 tiles while their grid is at most two
  // rounds of CUs (ViT-B/16 at 8 images: qkv 13.2 -> 11.7 us, out_proj 14.1 -> 11.9 us;
  // profiles/r03c/vit_gemm_ab.txt)
  if (M < 4096 && (long long)((M + 63) / 64) * (N / 128) <= 2LL * num_cus()) return 7;
  if (M >= 4096 && N % 256 == 0) {
    // 256- vs 192-row tiles: fraction of the last round of CU slots each leaves busy
    const double cus = 256.0;
    // a big-tile grid under half the CUs (N = 512 at ~6k rows: CoCoOp at 1 image per step):
    // 128x128 tiles, 3x the blocks (B = 1 step: N = 512 GEMMs 1.06 + 0.52 + 0.22 -> 0.85 + 0.42
    // + 0.18 ms; N >= 1536 stay on the big tiles, which measured faster there)
    if (((M + 191) / 192) * (N / 256) < cus / 2) {
      // knob CLIPK_GEMM_SMALL64 (A/B): 64x128 tiles where the 128x128 grid is one round or less
      static int s64 = -1;
      if (s64 < 0) {
        const char* e = getenv("CLIPK_GEMM_SMALL64");
        s64 = e ? atoi(e) : 0;
      }
      if (s64 && ((M + 127) / 128) * (N / 128) <= num_cus()) return 7;
      return 0;
    }
    const double w256 = ((M + 255) / 256) * (N / 256) / cus, w192 = ((M + 191) / 192) * (N / 256) / cus;
    const double e256 = w256 / __builtin_ceil(w256), e192 = w192 / __builtin_ceil(w192);
    // 192-row tiles only for a clear quantisation win: N = 512 at 47k rows (0.72 -> 0.96 of the
    // last round busy) measured 4 % faster; N = 1536 (0.87 -> 0.96) 5 % slower
    // (profiles/r02p_gemm_tile_rows.txt)
    return e192 > e256 + 0.15 ? 6 : 1;
  }
  return 0;
}

static unsigned long long* g_stamp = nullptr;
static int g_stamp_on = -1;
unsigned long long* gemm_stamp_buf() {
  if (g_stamp_on < 0) g_stamp_on = getenv("CLIPK_GEMM_STAMP") ? 1 : 0;
  if (!g_stamp_on) return nullptr;
  if (!g_stamp) {
    const size_t bytes = (size_t)STAMP_BLOCKS * (STAMP_TILES * 3 + 4) * 8;
    if (hipMalloc((void**)&g_stamp, bytes) != hipSuccess) { g_stamp_on = 0; return nullptr; }
    (void)hipMemset(g_stamp, 0, bytes);
  }
  return g_stamp;
}

// Persistent launch above this many tiles (knob CLIPK_GEMM_PERSIST_MIN, default 2 x CUs)
static int persist_min(int cus) {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("CLIPK_GEMM_PERSIST_MIN");
    v = e ? atoi(e) : -1;
  }
  return v >= 0 ? v : 2 * cus;
}

// 4-slot ring for 128x128 grids of at most one tile per CU (knob CLIPK_GEMM_DEEP=0 turns it
// off): three K steps in flight instead of one. Same-box A/B (profiles/r02p_ab_deep_small.txt):
// ViT forward at 8 images 1.34 -> 1.26 ms, headline step 11.94 -> 11.76 ms; 1-image step
// 3.92 -> 3.51 ms (its N = 512 text GEMMs run on such grids too)
bool deep_small() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLIPK_GEMM_DEEP");
    v = e ? atoi(e) : 1;
  }
  return v != 0;
}

static int g_skew = -1;
int gemm_skew() {
  if (g_skew < 0) {
    const char* e = getenv("CLIPK_GEMM_SKEW");
    g_skew = e ? atoi(e) : 0;
  }
  return g_skew;
}
// Diagnostic filter (tools/lab/step_stamps.py): stamp only launches of one epilogue id and at
// least this many rows, so the buffer holds the last such launch of a whole train step
unsigned long long* gemm_stamp_for(int epi, int M) {
  static int fe = -2, fm = 0;
  if (fe == -2) {
    const char* e = getenv("CLIPK_GEMM_STAMP_EPI");
    const char* m = getenv("CLIPK_GEMM_STAMP_MINM");
    fe = e ? atoi(e) : -1;
    fm = m ? atoi(m) : 0;
  }
  if ((fe >= 0 && epi != fe) || M < fm) return nullptr;
  return gemm_stamp_buf();
}
// (knob CLIPK_GEMM_T96=0: the 128x128 deep ring instead, A/B)
bool gemm_t96() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLIPK_GEMM_T96");
    v = e ? atoi(e) : 1;
  }
  return v != 0;
}
static int g_num_cus = 0;
int num_cus() {
  if (!g_num_cus) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      g_num_cus = n;
    else
      g_num_cus = 256;
  }
  return g_num_cus;
}

int pp_grid(int nwg, int cus) {
  const int full = (cus / 8) * 8;
  const int need = (nwg + 7) / 8 * 8;
  if (CLIPK_GEMM_PP == 2) return need;  // one tile per block (A/B)
  return need < full ? need : full;
}

// (Round 4 built a "split tail" for the N = 512 GEMMs -- 256x256 tiles with the tiles past the
// first round cut in two K halves on paired blocks, the first half's fp32 partial handed over
// through a caller workspace -- and measured it slower on the headline step, 10.67 -> 11.39
// ms/step, profiles/r04e/ab_split_tail.txt; removed in round 5.)

template <typename T, typename TO, typename TX, int EPI, int LNM = 0>
static int launch_gemm(const GemmArgs& g, hipStream_t st) {
  const int cfg = pick_cfg(g.M, g.N, (int)sizeof(T));
  const_cast<GemmArgs&>(g).stamp = gemm_stamp_buf();
  if (g_skew < 0) {
    const char* e = getenv("CLIPK_GEMM_SKEW");
    g_skew = e ? atoi(e) : 0;
  }
  const_cast<GemmArgs&>(g).skew = g_skew;
  if constexpr (__is_same(T, float)) {
    const int nwg = ((g.M + 127) / 128) * (g.N / 128);
    hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 128, 128, 2, 2, false, GEMM_ROWB, 2, false, false, LNM>), dim3(nwg), dim3(256), 0, st, g);
  } else {
    if (cfg == 1 || cfg == 3) {
      const int nwg = ((g.M + 255) / 256) * (g.N / 256);
      const int cus = num_cus();
      if (try_pp<T, TO, TX, EPI, 256, LNM>(g, nwg, st)) {
      } else if (cfg == 1 && nwg > 2 * cus) {
        // persistent: one 8-wave block per CU, grid a multiple of 8 (XCD groups)
        const int grid = (cus / 8) * 8;
        hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 256, 256, 2, 4, true, GEMM_ROWB, 2, false, false, LNM>), dim3(grid), dim3(512), 0, st, g);
      } else {
        hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 256, 256, 2, 4, false, GEMM_ROWB, 2, false, false, LNM>), dim3(nwg), dim3(512), 0, st, g);
      }
    } else if (cfg == 6) {
      const int nwg = ((g.M + 191) / 192) * (g.N / 256);
      const int cus = num_cus();
      if (try_pp<T, TO, TX, EPI, 192, LNM>(g, nwg, st)) {
      } else if constexpr (CLIPK_GEMM_RING)  // 4-slot ring of 64-B K steps: three steps in flight
        hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 192, 256, 2, 4, false, 64, 4, false, false, LNM>), dim3(nwg), dim3(512), 0, st, g);
      else if (nwg > persist_min(cus))
        hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 192, 256, 2, 4, true, GEMM_ROWB, 2, false, false, LNM>), dim3((cus / 8) * 8), dim3(512), 0, st, g);
      else
        hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 192, 256, 2, 4, false, GEMM_ROWB, 2, false, false, LNM>), dim3(nwg), dim3(512), 0, st, g);
    } else if (cfg == 7) {
      // 64x128 (4 waves of 32x64): twice the 128x128 grid for the small-M ViT projections
      const int nwg = ((g.M + 63) / 64) * (g.N / 128);
      if (nwg <= num_cus() && deep_small())
        hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 64, 128, 2, 2, false, GEMM_ROWB, 4, false, false, LNM>),
                           dim3(nwg), dim3(256), 0, st, g);
      else
        hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 64, 128, 2, 2, false, GEMM_ROWB, 2, false, false, LNM>),
                           dim3(nwg), dim3(256), 0, st, g);
    } else if (cfg == 2) {
      const int nwg = ((g.M + 255) / 256) * (g.N / 128);
      hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 256, 128, 4, 2, false, GEMM_ROWB, 2, false, false, LNM>), dim3(nwg), dim3(512), 0, st, g);
    } else {
      const int nwg = ((g.M + 127) / 128) * (g.N / 128);
      if (nwg <= num_cus() && deep_small())  // one tile per CU: 4-slot ring (144 KiB LDS), knob
        hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 128, 128, 2, 2, false, GEMM_ROWB, 4, false, false, LNM>), dim3(nwg),
                           dim3(256), 0, st, g);
      else
        hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 128, 128, 2, 2, false, GEMM_ROWB, 2, false, false, LNM>), dim3(nwg), dim3(256), 0, st, g);
    }
  }
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

template <typename TS = f32s>
static int dispatch_split(int out_dtype, int epi, int aux_dtype, const GemmArgs& g, hipStream_t st) {
  if (out_dtype != CLIPK_F32) return CLIPK_EDTYPE;
  switch (epi) {
    case CLIPK_EPI_BIAS: return launch_gemm_split<CLIPK_EPI_BIAS, 0, TS>(g, st);
    case CLIPK_EPI_BIAS_RES: return launch_gemm_split<CLIPK_EPI_BIAS_RES, 0, TS>(g, st);
    case CLIPK_EPI_BIAS_QGELU: return launch_gemm_split<CLIPK_EPI_BIAS_QGELU, 0, TS>(g, st);
    case CLIPK_EPI_DQGELU:
      return aux_dtype == CLIPK_F32 ? launch_gemm_split<CLIPK_EPI_DQGELU, 0, TS>(g, st) : CLIPK_EDTYPE;
    case CLIPK_EPI_NONE: return launch_gemm_split<CLIPK_EPI_NONE, 0, TS>(g, st);
    case EPI_QGELU_D: return launch_gemm_split<EPI_QGELU_D, 0, TS>(g, st);
    case EPI_DMUL: return aux_dtype == CLIPK_F32 ? launch_gemm_split<EPI_DMUL, 0, TS>(g, st) : CLIPK_EDTYPE;
    default: return CLIPK_EINVAL;
  }
}

// weight W [N, K] fp32 -> CLIPK_SPLIT_SCALE * W as (hi, lo) fp16 parts, per 8 consecutive k:
// 8 hi then 8 lo (one thread per 8-element group)
__global__ __launch_bounds__(256) void split_pack_kernel(int N, int K, const float* __restrict__ W, int ldw,
                                                         f16* __restrict__ out) {
  const int kg = K / 8;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * kg) return;
  const int n = (int)(i / kg), g8 = (int)(i % kg);
  const float* src = W + (size_t)n * ldw + 8 * g8;
  f16x8 h, l;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float x = src[c] * CLIPK_SPLIT_SCALE;
    h[c] = (f16)x;
    l[c] = (f16)(x - (float)h[c]);
  }
  f16x8* dst = reinterpret_cast<f16x8*>(out + ((size_t)n * K + 8 * g8) * 2);
  dst[0] = h;
  dst[1] = l;
}

// CLIPK_A_QGELU launches: non-persistent 2-slot kernels of the tile the shape would get
template <typename T, typename TO, typename TX, int EPI>
static int launch_gemm_ag(const GemmArgs& g, hipStream_t st) {
  const int cfg = pick_cfg(g.M, g.N, (int)sizeof(T));
  if (cfg == 6) {
    const int nwg = ((g.M + 191) / 192) * (g.N / 256);
    hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 192, 256, 2, 4, false, GEMM_ROWB, 2, true>), dim3(nwg),
                       dim3(512), 0, st, g);
  } else if (g.N % 256 == 0 && g.M >= 4096) {
    const int nwg = ((g.M + 255) / 256) * (g.N / 256);
    hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 256, 256, 2, 4, false, GEMM_ROWB, 2, true>), dim3(nwg),
                       dim3(512), 0, st, g);
  } else {
    const int nwg = ((g.M + 127) / 128) * (g.N / 128);
    hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 128, 128, 2, 2, false, GEMM_ROWB, 2, true>), dim3(nwg),
                       dim3(256), 0, st, g);
  }
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

// dtype dispatch: (in, out, epi[, aux])
template <typename T>
static int dispatch_out(int out_dtype, int epi, int aux_dtype, const GemmArgs& g, hipStream_t st,
                        bool ag = false) {
  if (epi == CLIPK_EPI_BIAS_RES) {
    // residual stream in fp32, or (16-bit text residual) in the operand dtype for both res and out
    if constexpr (sizeof(T) == 2) {
      if (ag) {
        if (out_dtype == CLIPK_F32) return launch_gemm_ag<T, float, float, CLIPK_EPI_BIAS_RES>(g, st);
        if (out_dtype == DT<T>::id) return launch_gemm_ag<T, T, T, CLIPK_EPI_BIAS_RES>(g, st);
        return CLIPK_EDTYPE;
      }
    }
    if (ag) return CLIPK_EINVAL;
    if (out_dtype == CLIPK_F32) return launch_gemm<T, float, float, CLIPK_EPI_BIAS_RES>(g, st);
    if constexpr (sizeof(T) == 2) {
      if (out_dtype == DT<T>::id) return launch_gemm<T, T, T, CLIPK_EPI_BIAS_RES>(g, st);
    }
    return CLIPK_EDTYPE;
  }
  if (ag) return CLIPK_EINVAL;  // the A-operand QuickGELU is wired for the residual epilogue
  if (epi == CLIPK_EPI_DQGELU) {
    // backward: out in the grad dtype (== T), aux = forward pre-activation
    if (out_dtype != DT<T>::id) return CLIPK_EDTYPE;
    if (aux_dtype == CLIPK_F16) return launch_gemm<T, T, f16, CLIPK_EPI_DQGELU>(g, st);
    if (aux_dtype == CLIPK_BF16) return launch_gemm<T, T, bf16, CLIPK_EPI_DQGELU>(g, st);
    if (aux_dtype == CLIPK_F32) return launch_gemm<T, T, float, CLIPK_EPI_DQGELU>(g, st);
    return CLIPK_EDTYPE;
  }
  if (epi == EPI_DMUL) {  // backward with the saved derivative: out (grad dtype) = acc * aux
    if (out_dtype != DT<T>::id) return CLIPK_EDTYPE;
    if (aux_dtype == CLIPK_F16) return launch_gemm<T, T, f16, EPI_DMUL>(g, st);
    if (aux_dtype == CLIPK_BF16) return launch_gemm<T, T, bf16, EPI_DMUL>(g, st);
    if (aux_dtype == CLIPK_F32) return launch_gemm<T, T, float, EPI_DMUL>(g, st);
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
  if (epi == EPI_QGELU_D) {
    if (out_dtype == CLIPK_F32 && sizeof(T) != 4) return CLIPK_EDTYPE;
    CLIPK_OUTS(EPI_QGELU_D)
  }
  if (epi == CLIPK_EPI_NONE) { CLIPK_OUTS(CLIPK_EPI_NONE) }
#undef CLIPK_OUTS
  return CLIPK_EINVAL;
}

}  // namespace clipk

using namespace clipk;

extern "C" int clipk_gemm(int in_dtype, int out_dtype, int epi, int M, int N, int K,
                          const void* A, int lda, const void* B, int ldb,
                          const float* bias, const void* res, int ldr,
                          void* out, int ldo, void* out2, const void* aux, int aux_dtype,
                          int ldaux, void* stream) {
  if (!A || !B || !out) return CLIPK_EINVAL;
  const bool ag = (epi & CLIPK_A_QGELU) != 0;
  const bool deriv = (epi & CLIPK_QGELU_DERIV) != 0;
  const int spf = split_flags(epi);
  epi &= ~(CLIPK_A_QGELU | CLIPK_QGELU_DERIV | CLIPK_A_SPLIT | CLIPK_OUT_SPLIT | CLIPK_OUT2_SPLIT_GAMMA);
  const bool split = in_dtype == CLIPK_F32S || in_dtype == CLIPK_F32S16;
  if (spf && (!split || out_dtype != CLIPK_F32 || (spf & 4))) return CLIPK_EINVAL;
  if (ag && (in_dtype == CLIPK_F32 || split || epi != CLIPK_EPI_BIAS_RES)) return CLIPK_EINVAL;
  if (deriv && epi != CLIPK_EPI_BIAS_QGELU && epi != CLIPK_EPI_DQGELU) return CLIPK_EINVAL;
  if (M <= 0) return M == 0 ? CLIPK_OK : CLIPK_ESHAPE;
  const int esz = (in_dtype == CLIPK_F32 || split) ? 4 : 2;
  if (N <= 0 || K <= 0 || N % GEMM_NMIN != 0 || (K * esz) % GEMM_ROWB != 0) return CLIPK_ESHAPE;
  if (lda < K || ldb < K || (lda * esz) % 16 || (ldb * esz) % 16 || ldo < N || ldo % 4)
    return CLIPK_ESHAPE;
  // CLIPK_F32S(16): B is clipk_split_pack's output, whose rows are exactly K split elements apart
  if (split && ldb != K) return CLIPK_ESHAPE;
  if ((epi == CLIPK_EPI_BIAS || epi == CLIPK_EPI_BIAS_RES || epi == CLIPK_EPI_BIAS_QGELU) && !bias)
    return CLIPK_EINVAL;
  if (epi == CLIPK_EPI_BIAS_RES && (!res || ldr < N || ldr % 4)) return CLIPK_EINVAL;
  if (epi == CLIPK_EPI_DQGELU && (!aux || ldaux < N || ldaux % 4)) return CLIPK_EINVAL;
  GemmArgs g{(const char*)A, (const char*)B, M, N, K, lda, ldb, bias, res, ldr, out, ldo, out2, aux,
             ldaux, nullptr, 1, 0};
  hipStream_t st = (hipStream_t)stream;
  if (deriv) epi = epi == CLIPK_EPI_BIAS_QGELU ? EPI_QGELU_D : EPI_DMUL;
  if (spf) {
    if ((epi == CLIPK_EPI_DQGELU || epi == EPI_DMUL) && aux_dtype != CLIPK_F32) return CLIPK_EDTYPE;
    return presplit_launch(in_dtype == CLIPK_F32S16, spf, epi, 0, g, st);
  }
  switch (in_dtype) {
    case CLIPK_F16: return dispatch_out<f16>(out_dtype, epi, aux_dtype, g, st, ag);
    case CLIPK_BF16: return dispatch_out<bf16>(out_dtype, epi, aux_dtype, g, st, ag);
    case CLIPK_F32: return dispatch_out<float>(out_dtype, epi, aux_dtype, g, st);
    case CLIPK_F32S: return dispatch_split<f32s>(out_dtype, epi, aux_dtype, g, st);
    case CLIPK_F32S16: return dispatch_split<f32h>(out_dtype, epi, aux_dtype, g, st);
    default: return CLIPK_EDTYPE;
  }
}

// |W| limit of clipk_split_pack (include/clipk.h): the packed hi part CLIPK_SPLIT_SCALE * W must
// stay a finite fp16 (below 65504, which it then cannot round past)
constexpr float kSplitPackMax = 65504.0f / CLIPK_SPLIT_SCALE;

// The weight checks below report through one device word per call, allocated stream-ordered for
// that call (two host threads or streams checking weights at once each get their own word; a
// module-scope flag could be cleared by one between the other's kernel and its read-back).
// Any HIP failure maps to a negative status (CLIPK_EHIP), so no failed check reads as an answer.
template <typename Launch>
static int flag_check(hipStream_t st, int* answer, Launch&& launch) {
  int* flag = nullptr;
  int h = 0;
  if (hipMallocAsync((void**)&flag, sizeof(int), st) != hipSuccess) return CLIPK_EHIP;
  hipError_t e = hipMemsetAsync(flag, 0, sizeof(int), st);
  if (e == hipSuccess) {
    launch(flag);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(&h, flag, sizeof(int), hipMemcpyDeviceToHost, st);
  const hipError_t ef = hipFreeAsync(flag, st);
  if (e == hipSuccess) e = ef;
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return CLIPK_EHIP;
  *answer = h;
  return CLIPK_OK;
}

// one pass: *flag = 1 when any |W| >= kSplitPackMax or W is not finite (the pack's output
// would hold an inf / NaN part)
__global__ __launch_bounds__(256) void split_range_kernel(int N, int K, const float* __restrict__ W, int ldw,
                                                          int* __restrict__ flag) {
  const long n = (long)N * K;
  bool bad = false;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float x = W[(i / K) * ldw + i % K];
    bad |= !(fabsf(x) < kSplitPackMax);  // NaN compares false
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) *flag = 1;
}

static unsigned check_grid(long n) {
  const long nb = (n + 255) / 256;
  return (unsigned)(nb < 1024 ? nb : 1024);
}

extern "C" int clipk_split_pack(int N, int K, const float* W, int ldw, void* out, void* stream) {
  if (!W || !out) return CLIPK_EINVAL;
  if (N <= 0 || K <= 0 || K % 32 != 0 || ldw < K) return CLIPK_ESHAPE;
  // the range precondition is enforced here, not left to the caller: one synchronous check
  // (packing runs once per model, at construction)
  const hipStream_t st = (hipStream_t)stream;
  int bad = 0;
  const int rc = flag_check(st, &bad, [&](int* flag) {
    hipLaunchKernelGGL(split_range_kernel, dim3(check_grid((long)N * K)), dim3(256), 0, st, N, K, W, ldw, flag);
  });
  if (rc != CLIPK_OK) return rc;
  if (bad) return CLIPK_ERANGE;
  const long n = (long)N * (K / 8);
  hipLaunchKernelGGL(split_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, N, K, W, ldw, (f16*)out);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

// *flag = 1 when any lo part of a packed weight is nonzero (per 8 k: 16 B hi, then 16 B lo);
// hi16 != null: also copy the hi parts to the compact fp16 [N, K] weight (clipk_split_hi16)
__global__ __launch_bounds__(256) void split_lo_kernel(long ngroups, const u32x4* __restrict__ packed,
                                                       u32x4* __restrict__ hi16, int* __restrict__ flag) {
  bool nz = false;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < ngroups; i += (long)gridDim.x * 256) {
    const u32x4 lo = packed[2 * i + 1];
    nz |= ((lo[0] | lo[1] | lo[2] | lo[3]) & 0x7fff7fffu) != 0;  // -0 counts as zero
    if (hi16) hi16[i] = packed[2 * i];
  }
  if (__any(nz) && (threadIdx.x & 63) == 0) *flag = 1;
}

extern "C" int clipk_split_lo_zero(int N, int K, const void* packed, int* result, void* stream) {
  if (!packed || !result) return CLIPK_EINVAL;
  if (N <= 0 || K <= 0 || K % 32 != 0) return CLIPK_ESHAPE;
  const hipStream_t st = (hipStream_t)stream;
  const long ng = (long)N * (K / 8);
  int nz = 0;
  const int rc = flag_check(st, &nz, [&](int* flag) {
    hipLaunchKernelGGL(split_lo_kernel, dim3(check_grid(ng)), dim3(256), 0, st, ng, (const u32x4*)packed,
                       (u32x4*)nullptr, flag);
  });
  if (rc != CLIPK_OK) return rc;
  *result = nz ? 0 : 1;
  return CLIPK_OK;
}

extern "C" int clipk_split_hi16(int N, int K, const void* packed, void* out, void* stream) {
  if (!packed || !out) return CLIPK_EINVAL;
  if (N <= 0 || K <= 0 || K % 32 != 0) return CLIPK_ESHAPE;
  const hipStream_t st = (hipStream_t)stream;
  const long ng = (long)N * (K / 8);
  int nz = 0;
  const int rc = flag_check(st, &nz, [&](int* flag) {
    hipLaunchKernelGGL(split_lo_kernel, dim3(check_grid(ng)), dim3(256), 0, st, ng, (const u32x4*)packed,
                       (u32x4*)out, flag);
  });
  if (rc != CLIPK_OK) return rc;
  return nz ? CLIPK_ERANGE : CLIPK_OK;  // a nonzero lo part: not fp16-valued (out unspecified)
}

namespace clipk {
template <typename T>
static int dispatch_ln(int epi, const GemmArgs& g, hipStream_t st) {
  if (!g.colsum) return launch_gemm<T, T, T, CLIPK_EPI_BIAS_RES, 1>(g, st);
  if (epi == CLIPK_EPI_BIAS) return launch_gemm<T, T, float, CLIPK_EPI_BIAS, 2>(g, st);
  if (epi == EPI_QGELU_D) return launch_gemm<T, T, float, EPI_QGELU_D, 2>(g, st);
  return launch_gemm<T, T, float, CLIPK_EPI_BIAS_QGELU, 2>(g, st);
}
// PREC fp32s (A fp32, B split-packed, fp32 out / residual / quickgelu')
template <typename TS>
static int dispatch_ln_split(int epi, const GemmArgs& g, hipStream_t st) {
  if (!g.colsum) return launch_gemm_split<CLIPK_EPI_BIAS_RES, 1, TS>(g, st);
  if (g.lngamma) {  // clipk_gemm_ln_gamma
    if (epi == CLIPK_EPI_BIAS) return launch_gemm_split<CLIPK_EPI_BIAS, 4, TS>(g, st);
    if (epi == EPI_QGELU_D) return launch_gemm_split<EPI_QGELU_D, 4, TS>(g, st);
    return launch_gemm_split<CLIPK_EPI_BIAS_QGELU, 4, TS>(g, st);
  }
  if (epi == CLIPK_EPI_BIAS) return launch_gemm_split<CLIPK_EPI_BIAS, 2, TS>(g, st);
  if (epi == EPI_QGELU_D) return launch_gemm_split<EPI_QGELU_D, 2, TS>(g, st);
  return launch_gemm_split<CLIPK_EPI_BIAS_QGELU, 2, TS>(g, st);
}
}  // namespace clipk

// LayerNorm folded into the text GEMMs (include/clipk.h): statistics partials out (EPI_BIAS_RES)
// or colsum + per-row (rstd, -rstd * mean) in (EPI_BIAS / EPI_BIAS_QGELU); 16-bit in and out, or
// CLIPK_F32S (fp32 A / out / residual, B split-packed).
extern "C" int clipk_gemm_ln(int in_dtype, int epi, int M, int N, int K, const void* A, int lda, const void* B,
                             int ldb, const float* bias, const void* res, int ldr, void* out, int ldo, void* out2,
                             float* stats, const float* colsum, const float* rnb, void* stream) {
  if (!A || !B || !out || !bias) return CLIPK_EINVAL;
  const bool split = in_dtype == CLIPK_F32S || in_dtype == CLIPK_F32S16;
  if (in_dtype != CLIPK_F16 && in_dtype != CLIPK_BF16 && !split) return CLIPK_EDTYPE;
  const bool deriv = (epi & CLIPK_QGELU_DERIV) != 0;  // fold form of c_fc: out2 = quickgelu'
  const int spf = split_flags(epi);
  epi &= ~(CLIPK_QGELU_DERIV | CLIPK_A_SPLIT | CLIPK_OUT_SPLIT | CLIPK_OUT2_SPLIT_GAMMA);
  // pre-split operands (PREC fp32s): A into the producer (c_proj reading c_fc's split output), the
  // fold's output split (c_fc -> c_proj); the gamma copy is clipk_gemm_ln_stats_split's
  if (spf && (!split || (spf & 4) || (!colsum && (spf & 2)) || (colsum && (spf & 1)))) return CLIPK_EINVAL;
  if (deriv && (epi != CLIPK_EPI_BIAS_QGELU || !colsum)) return CLIPK_EINVAL;
  if (!colsum) {  // producer: the statistics partials of the output
    if (!stats || rnb || epi != CLIPK_EPI_BIAS_RES || !res || ldr < N || ldr % 8) return CLIPK_EINVAL;
  } else {        // fold: (rstd, -rstd * mean) of A's rows in
    if (stats || !rnb || (epi != CLIPK_EPI_BIAS && epi != CLIPK_EPI_BIAS_QGELU)) return CLIPK_EINVAL;
  }
  if (M <= 0) return M == 0 ? CLIPK_OK : CLIPK_ESHAPE;
  const int esz = split ? 4 : 2;
  if (N <= 0 || K <= 0 || N % GEMM_NMIN != 0 || (K * esz) % GEMM_ROWB != 0) return CLIPK_ESHAPE;
  if (lda < K || ldb < K || lda % 8 || ldb % 8 || ldo < N || ldo % 8) return CLIPK_ESHAPE;
  if (split && ldb != K) return CLIPK_ESHAPE;  // clipk_split_pack's row stride
  GemmArgs g{(const char*)A, (const char*)B, M, N, K, lda, ldb, bias, res, ldr, out, ldo, out2, nullptr,
             0, nullptr, 1, 0, 0, stats, colsum, reinterpret_cast<const f32x2*>(rnb)};
  hipStream_t st = (hipStream_t)stream;
  if (deriv) epi = EPI_QGELU_D;
  if (spf) return presplit_launch(in_dtype == CLIPK_F32S16, spf, epi, colsum ? 2 : 1, g, st);
  if (in_dtype == CLIPK_F32S) return dispatch_ln_split<f32s>(epi, g, st);
  if (in_dtype == CLIPK_F32S16) return dispatch_ln_split<f32h>(epi, g, st);
  return in_dtype == CLIPK_F16 ? dispatch_ln<f16>(epi, g, st) : dispatch_ln<bf16>(epi, g, st);
}

// the statistics producer with the next fold's pre-split A as out2 (include/clipk.h; PREC fp32s,
// split mode 2)
extern "C" int clipk_gemm_ln_stats_split(int in_dtype, int epi, int M, int N, int K, const void* A, int lda,
                                         const void* B, int ldb, const float* bias, const void* res, int ldr,
                                         void* out, int ldo, float* stats, const float* gamma, void* out2,
                                         void* stream) {
  if (!A || !B || !out || !bias || !res || !stats || !gamma || !out2) return CLIPK_EINVAL;
  if (in_dtype != CLIPK_F32S16) return CLIPK_EDTYPE;
  const int spf = split_flags(epi) | 4;
  if ((epi & ~CLIPK_A_SPLIT) != CLIPK_EPI_BIAS_RES) return CLIPK_EINVAL;
  if (M <= 0) return M == 0 ? CLIPK_OK : CLIPK_ESHAPE;
  if (N <= 0 || K <= 0 || N % GEMM_NMIN != 0 || (K * 4) % GEMM_ROWB != 0) return CLIPK_ESHAPE;
  if (lda < K || ldb != K || lda % 8 || ldo < N || ldo % 8 || ldr < N || ldr % 8) return CLIPK_ESHAPE;
  GemmArgs g{(const char*)A, (const char*)B, M, N, K, lda, ldb, bias, res, ldr, out, ldo, out2, nullptr,
             0, nullptr, 1, 0, 0, stats, nullptr, nullptr};
  g.lngamma = gamma;
  return presplit_launch(true, spf, CLIPK_EPI_BIAS_RES, 1, g, (hipStream_t)stream);
}

// the fold with the LayerNorm weight on A (LNM 4; include/clipk.h): PREC fp32s only
extern "C" int clipk_gemm_ln_gamma(int in_dtype, int epi, int M, int N, int K, const void* A, int lda, const void* B,
                                   int ldb, const float* bias, void* out, int ldo, void* out2, const float* colsum,
                                   const float* rnb, const float* gamma, void* stream) {
  if (!A || !B || !out || !bias || !colsum || !rnb || !gamma) return CLIPK_EINVAL;
  if (in_dtype != CLIPK_F32S && in_dtype != CLIPK_F32S16) return CLIPK_EDTYPE;
  const bool deriv = (epi & CLIPK_QGELU_DERIV) != 0;
  const int spf = split_flags(epi);
  epi &= ~(CLIPK_QGELU_DERIV | CLIPK_A_SPLIT | CLIPK_OUT_SPLIT);
  if (spf & 4) return CLIPK_EINVAL;
  if (epi != CLIPK_EPI_BIAS && epi != CLIPK_EPI_BIAS_QGELU) return CLIPK_EINVAL;
  if (deriv && epi != CLIPK_EPI_BIAS_QGELU) return CLIPK_EINVAL;
  if (M <= 0) return M == 0 ? CLIPK_OK : CLIPK_ESHAPE;
  if (N <= 0 || K <= 0 || K > kGammaMax || N % GEMM_NMIN != 0 || (K * 4) % GEMM_ROWB != 0) return CLIPK_ESHAPE;
  if (lda < K || ldb != K || lda % 8 || ldo < N || ldo % 8) return CLIPK_ESHAPE;
  GemmArgs g{(const char*)A, (const char*)B, M, N, K, lda, ldb, bias, nullptr, 0, out, ldo, out2, nullptr,
             0, nullptr, 1, 0, 0, nullptr, colsum, reinterpret_cast<const f32x2*>(rnb)};
  g.lngamma = gamma;
  hipStream_t st = (hipStream_t)stream;
  if (deriv) epi = EPI_QGELU_D;
  if (spf) return presplit_launch(in_dtype == CLIPK_F32S16, spf, epi, 4, g, st);
  return in_dtype == CLIPK_F32S16 ? dispatch_ln_split<f32h>(epi, g, st) : dispatch_ln_split<f32s>(epi, g, st);
}

namespace clipk {
// clipk_gemm_ln_merge's in-kernel form: 16-bit, W = K = 512 (8 partials per row), the shape on the
// 192-row ping-pong tiles (the batch-1 text encoder's qkv / c_fc at 5.9k rows). Knob
// CLIPK_LN_MERGE_FUSED=0 (A/B): always the merge launch + clipk_gemm_ln.
static bool ln_merge_fused_ok(int in_dtype, int M, int N, int K) {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("CLIPK_LN_MERGE_FUSED");
    on = e ? atoi(e) : 1;
  }
  return on && CLIPK_GEMM_PP && (in_dtype == CLIPK_F16 || in_dtype == CLIPK_BF16) && K == 512 && N % 256 == 0 &&
         pick_cfg(M, N, 2) == 6;
}
template <typename T, int EPI>
static int launch_ln_merge(GemmArgs g, hipStream_t st) {
  g.stamp = gemm_stamp_buf();
  if (g_skew < 0) {
    const char* e = getenv("CLIPK_GEMM_SKEW");
    g_skew = e ? atoi(e) : 0;
  }
  g.skew = g_skew;
  const int nwg = ((g.M + 191) / 192) * (g.N / 256);
  hipLaunchKernelGGL((gemm_nt_kernel<T, T, float, EPI, 192, 256, 2, 4, true, GEMM_ROWB, 2, false, true, 3>),
                     dim3(pp_grid(nwg, num_cus())), dim3(512), 0, st, g);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}
template <typename T>
static int dispatch_ln_merge(int epi, const GemmArgs& g, hipStream_t st) {
  if (epi == CLIPK_EPI_BIAS) return launch_ln_merge<T, CLIPK_EPI_BIAS>(g, st);
  if (epi == EPI_QGELU_D) return launch_ln_merge<T, EPI_QGELU_D>(g, st);
  return launch_ln_merge<T, CLIPK_EPI_BIAS_QGELU>(g, st);
}
}  // namespace clipk

extern "C" int clipk_gemm_ln_merge_fused(int in_dtype, int M, int N, int K) {
  return ln_merge_fused_ok(in_dtype, M, N, K) ? 1 : 0;
}

// LayerNorm fold with the statistics merge (include/clipk.h): what clipk_ln_stats_merge +
// clipk_gemm_ln compute, in one launch where the shape allows (ln_merge_fused_ok), else those two.
extern "C" int clipk_gemm_ln_merge(int in_dtype, int epi, int M, int N, int K, const void* A, int lda, const void* B,
                                   int ldb, const float* bias, void* out, int ldo, void* out2, const float* stats,
                                   const float* colsum, float* mean, float* rstd, float* rnb, void* stream) {
  if (!stats || !colsum || !rnb) return CLIPK_EINVAL;
  if (M <= 0) return M == 0 ? CLIPK_OK : CLIPK_ESHAPE;  // (before the fused path: no zero-block launch)
  const int e0 = epi & ~CLIPK_QGELU_DERIV;
  if (!ln_merge_fused_ok(in_dtype, M, N, K) || lda < K || ldb < K || lda % 8 || ldb % 8 || ldo < N || ldo % 8 ||
      !A || !B || !out || !bias || (e0 != CLIPK_EPI_BIAS && e0 != CLIPK_EPI_BIAS_QGELU) ||
      ((epi & CLIPK_QGELU_DERIV) && e0 != CLIPK_EPI_BIAS_QGELU)) {
    // the two-launch form (it also reports every argument error)
    if (M > 0) {
      const int rc = clipk_ln_stats_merge(M, K, stats, mean, rstd, rnb, stream);
      if (rc != CLIPK_OK) return rc;
    }
    return clipk_gemm_ln(in_dtype, epi, M, N, K, A, lda, B, ldb, bias, nullptr, 0, out, ldo, out2, nullptr, colsum, rnb,
                         stream);
  }
  GemmArgs g{(const char*)A, (const char*)B, M, N, K, lda, ldb, bias, nullptr, 0, out, ldo, out2, nullptr,
             0, nullptr, 1, 0, 0, const_cast<float*>(stats), colsum, nullptr, mean, rstd,
             reinterpret_cast<f32x2*>(rnb)};
  hipStream_t st = (hipStream_t)stream;
  const int ee = (epi & CLIPK_QGELU_DERIV) ? EPI_QGELU_D : e0;
  return in_dtype == CLIPK_F16 ? dispatch_ln_merge<f16>(ee, g, st) : dispatch_ln_merge<bf16>(ee, g, st);
}

namespace clipk {
// Split-K finish: out = epi(sum_s part[s] + bias [+ res]) in a fixed slice order
// (deterministic), 4 columns per thread.
template <typename TO, int EPI>
__global__ __launch_bounds__(256) void splitk_finish_kernel(int S, int M, int N, const float* __restrict__ part,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ res, int ldr,
                                                            TO* __restrict__ out, int ldo, TO* __restrict__ out2) {
  const int n4 = N >> 2;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)M * n4) return;
  const int m = (int)(i / n4), c = (int)(i % n4) * 4;
  // the first 8 slices' loads all issued before the sums (clamped to valid slices: no load
  // behind a branch), summed in slice order
  constexpr int SB = 8;
  f32x4 t[SB];
#pragma unroll
  for (int s = 0; s < SB; ++s)
    t[s] = *reinterpret_cast<const f32x4*>(part + ((size_t)(s < S ? s : S - 1) * M + m) * N + c);
  f32x4 v = t[0];
#pragma unroll
  for (int s = 1; s < SB; ++s)
    if (s < S) v += t[s];
  for (int s = SB; s < S; ++s) v += *reinterpret_cast<const f32x4*>(part + ((size_t)s * M + m) * N + c);
  if constexpr (EPI != CLIPK_EPI_NONE) v += *reinterpret_cast<const f32x4*>(bias + c);
  if constexpr (EPI == CLIPK_EPI_BIAS_RES) v += *reinterpret_cast<const f32x4*>(res + (size_t)m * ldr + c);
  if constexpr (EPI == CLIPK_EPI_BIAS_QGELU) {
    if (out2) store4<TO>(out2 + (size_t)m * ldo + c, v[0], v[1], v[2], v[3]);
    v = (f32x4){quick_gelu(v[0]), quick_gelu(v[1]), quick_gelu(v[2]), quick_gelu(v[3])};
  }
  if constexpr (EPI == EPI_QGELU_D) {
    if (out2)
      store4<TO>(out2 + (size_t)m * ldo + c, quick_gelu_grad(v[0]), quick_gelu_grad(v[1]), quick_gelu_grad(v[2]),
                 quick_gelu_grad(v[3]));
    v = (f32x4){quick_gelu(v[0]), quick_gelu(v[1]), quick_gelu(v[2]), quick_gelu(v[3])};
  }
  store4<TO>(out + (size_t)m * ldo + c, v[0], v[1], v[2], v[3]);
}

// Slices for a GEMM whose 128x128 tile grid would leave most CUs idle (small M): only when
// the grid covers under half of the CUs (the ViT's N = 768 projections at B = 8: 78 tiles;
// grids of 234-312 tiles measured no better split), enough slices for ~2 blocks per CU,
// each slice >= 8 K steps, at most 8 slices.
static int auto_splits(int M, int N, int K, int esz, int tile_rows = 128) {
  if (M <= 0 || N % GEMM_NMIN) return 1;
  const int tiles = ((M + tile_rows - 1) / tile_rows) * (N / 128);
  if (2 * tiles >= num_cus()) return 1;
  const int nk = K * esz / GEMM_ROWB;
  int s = (2 * num_cus()) / tiles;  // slices x tiles within one round of 2 blocks per CU
  s = s > 8 ? 8 : s;
  s = s > nk / 8 ? nk / 8 : s;  // >= 8 K steps per slice: the ViT's K = 768 c_proj measured
                                // 11.6 us unsplit vs 17.4 us in 3 slices + finish
  return s < 1 ? 1 : s;
}
}  // namespace clipk

extern "C" int clipk_gemm_auto_splits(int in_dtype, int M, int N, int K) {
  // fp32s small-M GEMMs run 64x128 tiles (launch_gemm_split): their grid is the one to fill
  if (in_dtype == CLIPK_F32S || in_dtype == CLIPK_F32S16) return auto_splits(M, N, K, 4, M < 4096 ? 64 : 128);
  return auto_splits(M, N, K, in_dtype == CLIPK_F32 ? 4 : 2);
}

extern "C" size_t clipk_gemm_splitk_ws_bytes(int M, int N, int splits) {
  if (M <= 0 || N <= 0 || splits <= 1) return 0;
  return (size_t)splits * M * N * sizeof(float);
}

template <typename TO, int EPI>
static int splitk_finish(int S, const GemmArgs& g, const float* part, hipStream_t st) {
  const long n = (long)g.M * (g.N / 4);
  hipLaunchKernelGGL((splitk_finish_kernel<TO, EPI>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, S, g.M,
                     g.N, part, g.bias, (const float*)g.res, g.ldr, (TO*)g.out, g.ldo, (TO*)g.out2);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_gemm_splitk(int in_dtype, int out_dtype, int epi, int M, int N, int K,
                                 const void* A, int lda, const void* B, int ldb,
                                 const float* bias, const void* res, int ldr,
                                 void* out, int ldo, void* out2, int splits, void* ws, size_t ws_bytes,
                                 void* stream) {
  const bool split = in_dtype == CLIPK_F32S || in_dtype == CLIPK_F32S16;
  const int esz = (in_dtype == CLIPK_F32 || split) ? 4 : 2;
  if (splits <= 0) splits = clipk_gemm_auto_splits(in_dtype, M, N, K);
  if (splits <= 1 || M <= 0)
    return clipk_gemm(in_dtype, out_dtype, epi, M, N, K, A, lda, B, ldb, bias, res, ldr, out, ldo, out2,
                      nullptr, 0, 0, stream);
  if (!A || !B || !out || !ws) return CLIPK_EINVAL;
  if (N <= 0 || K <= 0 || N % GEMM_NMIN != 0 || (K * esz) % GEMM_ROWB != 0) return CLIPK_ESHAPE;
  if (lda < K || ldb < K || (lda * esz) % 16 || (ldb * esz) % 16 || ldo < N || ldo % 4) return CLIPK_ESHAPE;
  if (splits > K * esz / GEMM_ROWB) return CLIPK_ESHAPE;
  if (split && ldb != K) return CLIPK_ESHAPE;  // clipk_split_pack's row stride
  const bool deriv = (epi & CLIPK_QGELU_DERIV) != 0;
  epi &= ~CLIPK_QGELU_DERIV;
  if (epi == CLIPK_EPI_DQGELU || (deriv && epi != CLIPK_EPI_BIAS_QGELU)) return CLIPK_EINVAL;
  if ((epi == CLIPK_EPI_BIAS || epi == CLIPK_EPI_BIAS_RES || epi == CLIPK_EPI_BIAS_QGELU) && !bias)
    return CLIPK_EINVAL;
  if (epi == CLIPK_EPI_BIAS_RES && (!res || ldr < N || ldr % 4 || out_dtype != CLIPK_F32)) return CLIPK_EINVAL;
  if (ws_bytes < clipk_gemm_splitk_ws_bytes(M, N, splits)) return CLIPK_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  // slices: EPI_NONE fp32 partials [splits][M][N] (128x128 tiles, one block per tile and slice)
  GemmArgs p{(const char*)A, (const char*)B, M, N, K, lda, ldb, nullptr, nullptr, 0, ws, N, nullptr, nullptr, 0,
             gemm_stamp_buf(), splits, (long long)M * N};
  const int nwg = ((M + 127) / 128) * (N / 128) * splits;
  switch (in_dtype) {
    case CLIPK_F16:
      hipLaunchKernelGGL((gemm_nt_kernel<f16, float, float, CLIPK_EPI_NONE, 128, 128, 2, 2, false>), dim3(nwg),
                         dim3(256), 0, st, p);
      break;
    case CLIPK_BF16:
      hipLaunchKernelGGL((gemm_nt_kernel<bf16, float, float, CLIPK_EPI_NONE, 128, 128, 2, 2, false>), dim3(nwg),
                         dim3(256), 0, st, p);
      break;
    case CLIPK_F32:
      hipLaunchKernelGGL((gemm_nt_kernel<float, float, float, CLIPK_EPI_NONE, 128, 128, 2, 2, false>), dim3(nwg),
                         dim3(256), 0, st, p);
      break;
    case CLIPK_F32S:  // slice partials already carry the 1 / CLIPK_SPLIT_SCALE (EPI_NONE epilogue)
      hipLaunchKernelGGL((gemm_nt_kernel<f32s, float, float, CLIPK_EPI_NONE, 128, 128, 2, 2, false>), dim3(nwg),
                         dim3(256), 0, st, p);
      break;
    case CLIPK_F32S16:
      hipLaunchKernelGGL((gemm_nt_kernel<f32h, float, float, CLIPK_EPI_NONE, 128, 128, 2, 2, false>), dim3(nwg),
                         dim3(256), 0, st, p);
      break;
    default: return CLIPK_EDTYPE;
  }
  CLIPK_CHECK_LAUNCH();
  GemmArgs g{(const char*)A, (const char*)B, M, N, K, lda, ldb, bias, res, ldr, out, ldo, out2, nullptr, 0,
             nullptr, 1, 0};
  const float* part = (const float*)ws;  // the finish pass reads an fp32 residual (checked above)
#define CLIPK_FIN(EPIV)                                                           \
  switch (out_dtype) {                                                            \
    case CLIPK_F32: return splitk_finish<float, EPIV>(splits, g, part, st);      \
    case CLIPK_F16: return splitk_finish<f16, EPIV>(splits, g, part, st);        \
    case CLIPK_BF16: return splitk_finish<bf16, EPIV>(splits, g, part, st);      \
    default: return CLIPK_EDTYPE;                                                 \
  }
  if (epi == CLIPK_EPI_NONE) { CLIPK_FIN(CLIPK_EPI_NONE) }
  if (epi == CLIPK_EPI_BIAS) { CLIPK_FIN(CLIPK_EPI_BIAS) }
  if (epi == CLIPK_EPI_BIAS_QGELU && deriv) { CLIPK_FIN(EPI_QGELU_D) }
  if (epi == CLIPK_EPI_BIAS_QGELU) { CLIPK_FIN(CLIPK_EPI_BIAS_QGELU) }
  if (epi == CLIPK_EPI_BIAS_RES) return splitk_finish<float, CLIPK_EPI_BIAS_RES>(splits, g, part, st);
#undef CLIPK_FIN
  return CLIPK_EINVAL;
}

// Diagnostic: copy the per-block stamps of the last launch (CLIPK_GEMM_STAMP set) to host
// [STAMP_BLOCKS][4 + 3 * STAMP_TILES] u64: memtime0, realtime0, then per tile
// (k-loop start, k-loop end, epilogue end) s_memrealtime (100 MHz), then memtime / realtime
// at the block's end (effective shader clock).
extern "C" int clipk_gemm_stamps(void* host, size_t bytes) {
  const size_t need = (size_t)STAMP_BLOCKS * (STAMP_TILES * 3 + 4) * 8;
  if (!g_stamp || !host || bytes < need) return CLIPK_EINVAL;
  if (hipDeviceSynchronize() != hipSuccess) return (int)hipGetLastError();
  if (hipMemcpy(host, g_stamp, need, hipMemcpyDeviceToHost) != hipSuccess) return (int)hipGetLastError();
  return CLIPK_OK;
}

// Benchmark knob: force a tile configuration (-1 = automatic choice).
extern "C" int clipk_gemm_set_config(int cfg) {
  if (cfg < -1 || cfg > 7 || cfg == 4 || cfg == 5) return CLIPK_EINVAL;
  g_force_cfg = cfg;
  return CLIPK_OK;
}
