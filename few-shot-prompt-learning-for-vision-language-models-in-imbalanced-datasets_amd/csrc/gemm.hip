// MFMA GEMM with fused epilogues for every linear layer on the CoOp/CoCoOp path:
//   out[M,N] = epilogue( A[M,K] . B[N,K]^T ),  fp32 accumulate.
// A = activations (row-major, K contiguous), B = packed frozen weight (row-major [N,K]),
// i.e. the nn.Linear layout (PromptSRC/clip/model.py:171-177) and its transpose for
// the input-grad GEMMs (pre-packed once, so backward is the same "NT" form).
//
// gfx950 design:
//  * Block tiles 256x256 / 256x128 (8 waves) for the large-M text GEMMs, 128x128
//    (4 waves) otherwise; K staged 128 bytes per row (64 halfs or 32 floats) into a 2-stage
//    LDS ring by global_load_lds_dwordx4 (glds): one wave-instruction = 8 rows x 128 B
//    = 1 KiB, lane-linear in LDS.
//  * LDS image row-swizzled on the SOURCE address (glds writes lane-linear): physical
//    16-B chunk p = c ^ ((row >> 1) & 7). With rows = lane&15 read by ds_read_b128 this
//    puts each 16-lane group on 16 distinct 16-B slots of the 256-B bank row (no conflict).
//  * MFMA v_mfma_f32_16x16x32_{f16,bf16} (or v_mfma_f32_16x16x4_f32 for the fp32 parity
//    mode) with SWAPPED operands (weights as the A operand): each lane then holds 4
//    consecutive output columns of one row, so the epilogue issues 8/16-B row stores and
//    float4 bias/residual loads.
//  * XCD-aware bijective block remap: consecutive tiles of one A row-panel run on one XCD
//    so the panel is fetched from HBM once and re-read from that XCD's L2.
#include <cstdlib>

#include "common.h"

namespace clipk {

constexpr int GEMM_ROWB = 128;  // bytes per staged row (BK = 64 halfs / 32 floats)
constexpr int GEMM_NMIN = 128;  // N granularity accepted by the C-ABI
constexpr int EPI_SCRATCH = 16 * 64 * 4;  // per-wave epilogue transpose tile [16][64] fp32

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

// Raw register type of one lane's 4 epilogue operand values (residual f32, aux TX).
template <int EPI, typename TX> struct ExtRaw { typedef f32x4 type; };
template <> struct ExtRaw<CLIPK_EPI_DQGELU, f16> { typedef uint2 type; };
template <> struct ExtRaw<CLIPK_EPI_DQGELU, bf16> { typedef uint2 type; };

__device__ __forceinline__ f32x4 ext_f32(f32x4 v) { return v; }
template <typename TX> __device__ __forceinline__ f32x4 ext_f32(f32x4 v) { return v; }
template <typename TX> __device__ __forceinline__ f32x4 ext_f32(uint2 v) {
  float o[4];
  load4<TX>(reinterpret_cast<const TX*>(&v), o);
  return (f32x4){o[0], o[1], o[2], o[3]};
}

// Block tile BM x BN, WM x WN waves (each (BM/WM) x (BN/WN) = TM x TN 16x16 sub-tiles),
// 2-stage LDS ring, one barrier per 128-byte K step. PERSIST: the grid is sized to the
// CU count and each block walks an XCD-contiguous run of tiles; the last K step of a tile
// prefetches the first stage of the next tile, so that load overlaps the epilogue.
template <typename T, typename TO, typename TX, int EPI, int BM, int BN, int WM, int WN, bool PERSIST>
__global__ __launch_bounds__(WM * WN * 64, 2) void gemm_nt_kernel(GemmArgs g) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int OPA = BM * GEMM_ROWB, OPB = BN * GEMM_ROWB, STAGE = OPA + OPB;
  constexpr int IA = BM / 8 / NW, IB = BN / 8 / NW;  // glds (8 rows x 128 B) per wave per stage
  static_assert(IA >= 1 && IB >= 1 && BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile/wave mismatch");
  __shared__ CLIPK_LDS_ALIGN char smem[2 * STAGE + NW * EPI_SCRATCH];  // one array (see header)
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // ---- XCD-aware bijective tile split: XCD group x owns tiles [t_beg, t_end) (row-panel
  // major, so the tiles sharing an A panel run on one XCD and re-read it from its L2).
  const int ntn = g.N / BN;
  const int ntm = (g.M + BM - 1) / BM;
  const int nwg = ntm * ntn;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int t_beg = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int t_end = t_beg + (xcd < r ? q + 1 : q);
  const int t_step = PERSIST ? (int)(gridDim.x >> 3) : 1;
  int tile = t_beg + (bid >> 3);
  if (tile >= t_end) return;  // block-uniform

  const size_t esz = sizeof(T);
  const int nk = (int)((size_t)g.K * esz / GEMM_ROWB);
  const char* srcA[IA];
  const char* srcB[IB];
  auto set_tile = [&](int t) {
    const int tm0 = (t / ntn) * BM, tn0 = (t % ntn) * BN;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int row = (w * IA + i) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);  // source-side swizzle
      int ga = tm0 + row;
      ga = ga < g.M ? ga : g.M - 1;
      srcA[i] = g.A + ((size_t)ga * g.lda) * esz + c * 16;
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int row = (w * IB + i) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      srcB[i] = g.B + ((size_t)(tn0 + row) * g.ldb) * esz + c * 16;
    }
  };
  auto stage = [&](int s, int kt) {
    char* base = smem + s * STAGE;
    const size_t koff = (size_t)kt * GEMM_ROWB;
#pragma unroll
    for (int i = 0; i < IA; ++i) glds16(srcA[i] + koff, base + (w * IA + i) * 8 * GEMM_ROWB);
#pragma unroll
    for (int i = 0; i < IB; ++i) glds16(srcB[i] + koff, base + OPA + (w * IB + i) * 8 * GEMM_ROWB);
  };

  const int wm = w / WN, wn = w % WN;
  const int fr = lane & 15;         // fragment row within a 16-row sub-tile
  const int fq = lane >> 4;         // 16-B chunk within a 64-B k-window
  const int sw = (fr >> 1) & 7;     // row swizzle (sub-tile row base is a multiple of 16)
  constexpr bool HAS_BIAS = EPI == CLIPK_EPI_BIAS || EPI == CLIPK_EPI_BIAS_RES || EPI == CLIPK_EPI_BIAS_QGELU;
  constexpr bool HAS_EXT = EPI == CLIPK_EPI_BIAS_RES || EPI == CLIPK_EPI_DQGELU;

  set_tile(tile);
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int it = 0;  // global K-step counter (LDS buffer = it & 1)

  while (true) {
    const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
    const int next = tile + t_step;
    const bool has_next = PERSIST && next < t_end;
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    const int nbase = n0 + wn * (BN / WN);
    const int er = lane >> 4, ec = lane & 15;  // read-back: row er of each 4-row step, chunk ec
    const int ncol = nbase + 4 * ec;
    // residual / aux operands of group i+1 are loaded while group i is transposed and
    // stored (raw, converted at use: a conversion right after the load would wait for it)
    typedef typename ExtRaw<EPI, TX>::type XR;
    XR ext_nxt[4];
    auto load_ext = [&](int i, XR* dst) {
      if constexpr (HAS_EXT) {
        const int mg = m0 + wm * (BM / WM) + i * 16;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          int mc = mg + 4 * q + er;
          mc = mc < g.M ? mc : g.M - 1;
          if constexpr (EPI == CLIPK_EPI_BIAS_RES)
            dst[q] = *reinterpret_cast<const XR*>(g.res + (size_t)mc * g.ldr + ncol);
          else
            dst[q] = *reinterpret_cast<const XR*>((const TX*)g.aux + (size_t)mc * g.ldaux + ncol);
        }
      }
    };
    // group 0's operands are loaded at the top of the last K step (its MFMAs hide them)
    for (int kt = 0; kt < nk; ++kt, ++it) {
      const int cur = it & 1;
      const bool last = kt + 1 == nk;
      if (!last) {
        stage(cur ^ 1, kt + 1);
      } else if (has_next) {
        set_tile(next);
        stage(cur ^ 1, 0);  // next tile's first stage flies during this tile's epilogue
      }
      if (last) load_ext(0, ext_nxt);
      const char* As = smem + cur * STAGE + (wm * (BM / WM) + fr) * GEMM_ROWB;
      const char* Bs = smem + cur * STAGE + OPA + (wn * (BN / WN) + fr) * GEMM_ROWB;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int p = ((kk * 4 + fq) ^ sw) * 16;
        u32x4 a[TM], b[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = *reinterpret_cast<const u32x4*>(Bs + j * 16 * GEMM_ROWB + p);
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = *reinterpret_cast<const u32x4*>(As + i * 16 * GEMM_ROWB + p);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma<T>(b[j], a[i], acc[i][j]);
      }
      if (!last) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }

    // ---- epilogue through a per-wave LDS scratch [16][64] fp32: the MFMA layout (lane =
    // row fr, 4 columns per sub-tile) is transposed to row-major so that each store / residual
    // / aux access instruction covers 4 rows x full 64-column runs (128 B of f16, 256 B of
    // f32) instead of 16 rows x 32 B. 16-B chunk c of row r sits at chunk c ^ r (conflict-free
    // on both the write and the read-back side).
    static_assert(TN == 4, "epilogue transpose assumes 64 columns per wave");
    f32x4 bia = {0.f, 0.f, 0.f, 0.f};
    if constexpr (HAS_BIAS) bia = *reinterpret_cast<const f32x4*>(g.bias + ncol);
    float* scr = reinterpret_cast<float*>(smem + 2 * STAGE + w * EPI_SCRATCH);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int mg = m0 + wm * (BM / WM) + i * 16;  // first row of this 16-row group
      XR ext[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) ext[q] = ext_nxt[q];
      if (i + 1 < TM) load_ext(i + 1, ext_nxt);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // previous group's read-back done
#pragma unroll
      for (int j = 0; j < TN; ++j)
        *reinterpret_cast<f32x4*>(scr + fr * 64 + (((4 * j + fq) ^ fr) << 2)) = acc[i][j];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private: no barrier needed
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rr = 4 * q + er;
        const int m = mg + rr;
        f32x4 v = *reinterpret_cast<const f32x4*>(scr + rr * 64 + ((ec ^ rr) << 2));
        if (m >= g.M) continue;
        if constexpr (HAS_BIAS) v += bia;
        if constexpr (EPI == CLIPK_EPI_BIAS_RES) {
          *reinterpret_cast<f32x4*>((float*)g.out + (size_t)m * g.ldo + ncol) = v + ext_f32(ext[q]);
        } else if constexpr (EPI == CLIPK_EPI_BIAS_QGELU) {
          if (g.out2) store4<TO>((TO*)g.out2 + (size_t)m * g.ldo + ncol, v[0], v[1], v[2], v[3]);
          store4<TO>((TO*)g.out + (size_t)m * g.ldo + ncol, quick_gelu(v[0]), quick_gelu(v[1]),
                     quick_gelu(v[2]), quick_gelu(v[3]));
        } else if constexpr (EPI == CLIPK_EPI_DQGELU) {
          const f32x4 hv = ext_f32<TX>(ext[q]);
          store4<TO>((TO*)g.out + (size_t)m * g.ldo + ncol, v[0] * quick_gelu_grad(hv[0]),
                     v[1] * quick_gelu_grad(hv[1]), v[2] * quick_gelu_grad(hv[2]),
                     v[3] * quick_gelu_grad(hv[3]));
        } else {
          store4<TO>((TO*)g.out + (size_t)m * g.ldo + ncol, v[0], v[1], v[2], v[3]);
        }
      }
    }
    if (!has_next) break;
    tile = next;
    // the K loop left `it` one past this tile's last step: buffer it & 1 holds the
    // next tile's prefetched first stage
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

// Tile configurations: 0 = 128x128 (4 waves, 64 KiB LDS, 2 blocks/CU),
// 1 = 256x256 (8 waves, 128 KiB, persistent when the grid exceeds 2 waves of CUs),
// 2 = 256x128 (8 waves, 96 KiB), 3 = 256x256 non-persistent (benchmark knob).
static int g_force_cfg = -2;  // -2: unread, -1: auto
static int pick_cfg(int M, int N, int esz) {
  if (g_force_cfg == -2) {
    const char* e = getenv("CLIPK_GEMM_CFG");
    g_force_cfg = e ? atoi(e) : -1;
  }
  if (esz == 4) return 0;  // fp32 parity path: one configuration
  if (g_force_cfg >= 0) {
    if ((g_force_cfg == 1 || g_force_cfg == 3) && N % 256 == 0) return g_force_cfg;
    if (g_force_cfg == 2) return 2;
    return 0;
  }
  if (M >= 4096 && N % 256 == 0) return 1;  // measured best for every text GEMM shape
  return 0;
}

static int g_num_cus = 0;
static int num_cus() {
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

template <typename T, typename TO, typename TX, int EPI>
static int launch_gemm(const GemmArgs& g, hipStream_t st) {
  const int cfg = pick_cfg(g.M, g.N, (int)sizeof(T));
  if constexpr (sizeof(T) == 4) {
    const int nwg = ((g.M + 127) / 128) * (g.N / 128);
    hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 128, 128, 2, 2, false>), dim3(nwg), dim3(256), 0, st, g);
  } else {
    if (cfg == 1 || cfg == 3) {
      const int nwg = ((g.M + 255) / 256) * (g.N / 256);
      const int cus = num_cus();
      if (cfg == 1 && nwg > 2 * cus) {
        // persistent: one 8-wave block per CU, grid a multiple of 8 (XCD groups)
        const int grid = (cus / 8) * 8;
        hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 256, 256, 2, 4, true>), dim3(grid), dim3(512), 0, st, g);
      } else {
        hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 256, 256, 2, 4, false>), dim3(nwg), dim3(512), 0, st, g);
      }
    } else if (cfg == 2) {
      const int nwg = ((g.M + 255) / 256) * (g.N / 128);
      hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 256, 128, 4, 2, false>), dim3(nwg), dim3(512), 0, st, g);
    } else {
      const int nwg = ((g.M + 127) / 128) * (g.N / 128);
      hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, 128, 128, 2, 2, false>), dim3(nwg), dim3(256), 0, st, g);
    }
  }
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
  if (N <= 0 || K <= 0 || N % GEMM_NMIN != 0 || (K * esz) % GEMM_ROWB != 0) return CLIPK_ESHAPE;
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

// Benchmark knob: force a tile configuration (-1 = automatic choice).
extern "C" int clipk_gemm_set_config(int cfg) {
  if (cfg < -1 || cfg > 3) return CLIPK_EINVAL;
  g_force_cfg = cfg;
  return CLIPK_OK;
}
