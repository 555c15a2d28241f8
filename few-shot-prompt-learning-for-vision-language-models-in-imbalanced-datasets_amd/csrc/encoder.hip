// Native encoder runtime: the per-layer launch sequences of the CLIP text transformer
// (forward + input-grad backward) and of the ViT (forward only), behind an opaque
// handle that holds host-side pointer tables to caller-owned packed weights.
//
// Replaces the Python layer loop of Transformer.forward (PromptSRC/clip/model.py:361-367)
// driven by TextEncoder.forward (trainers/coop.py:195-205) / VisionTransformer.forward
// (model.py:401-431), and torch autograd's backward through the frozen text encoder.
// All launches go to the caller's stream; no allocation, no host sync (graph-capturable).
#include <vector>
#include <array>
#include <cstring>
#include <new>
#include <cstdlib>
#include <algorithm>

#include "common.h"

// Deep prompts (IVLP / MaPLe / PromptSRC, model.py:191-331): before layer l in 1..n_deep the
// rows rows[p * n_per + i] of the residual stream are replaced by prompt row p of
// prompts[l-1] ([n_deep][n_ctx][W] fp32); the backward sums the gradient of those rows into
// grads[l-1] and zeroes them (the replaced rows' previous values reach nothing).
struct DeepPrompts {
  int n_deep = 0, n_ctx = 0, n_per = 0;
  const int* rows = nullptr;
  const float* prompts = nullptr;
  float* grads = nullptr;
};

struct clipk_encoder {
  int kind;  // 0 text, 1 vision
  int W, layers, heads, E, act, grad;
  int res, patch, Kp, Limg;
  std::vector<std::array<const void*, 16>> lw;
  std::array<const void*, 8> head;
  DeepPrompts deep;
  // clipk_encoder_set_input_rows: 1 = on the shared-prefix packed layout only the P prefix rows
  // of each group carry per-group (trainable) values; the class rows of x0 are the same for
  // every group and their input gradient is not wanted
  int prefix_input = 0;
  // clipk_encoder_set_ln_fold: per layer {W_in', s_in, c_in, W_fc', s_fc, c_fc} (empty: off)
  std::vector<std::array<const void*, 6>> fold;
  // clipk_encoder_set_split: PREC fp32s -- fp32 activations, every GEMM weight split-packed
  // (clipk_split_pack) and every GEMM on the split-fp16 MFMA path (CLIPK_F32S); 2: the weights
  // given at creation are fp16-valued (clipk_split_lo_zero), their GEMMs run CLIPK_F32S16; the
  // LayerNorm fold then takes W itself and applies gamma to A (clipk_gemm_ln_gamma), so it runs
  // CLIPK_F32S16 too
  int split = 0;
  int split_target = 7;     // the backward's gradient scale puts max |s dtxt| in [2^(t-1), 2^t)
  int* status = nullptr;    // clipk_encoder_set_status: overflow flags of split calls (device)
};

namespace clipk {

static inline size_t esize(int dt) { return (dt == CLIPK_F32 || dt == CLIPK_F32S || dt == CLIPK_F32S16) ? 4 : 2; }

// PREC fp32s: while an encoder call of a split encoder runs, its fp32 GEMMs take the split-packed
// weights (CLIPK_F32S). Set per call (RAII, per host thread) by the entry points below, so the
// shared layer-loop code keeps passing the activation dtype.
static thread_local int t_split = 0;
struct SplitScope {
  int prev;
  explicit SplitScope(const clipk_encoder* e) : prev(t_split) { t_split = e->split; }
  ~SplitScope() { t_split = prev; }
};
static inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// Residual stream dtype of the TEXT encoder: the 16-bit activation dtype under PREC
// fp16/bf16 (CLIP's own fp16 semantics: the whole residual path in half precision, LN
// statistics in fp32), fp32 under PREC fp32. CLIPK_TEXT_RES32 forces fp32 (A/B knob).
static int res_dtype(const clipk_encoder* e) {
  static const bool force32 = getenv("CLIPK_TEXT_RES32") != nullptr;
  return (e->act == CLIPK_F32 || force32) ? CLIPK_F32 : e->act;
}

struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(void* b) : base((char*)b) {}
  void* take(size_t bytes) {
    void* p = base ? base + off : nullptr;
    off += align_up(bytes);
    return p;
  }
};

// ---------------------------------------------------------------- profiling (bench roofline)
// Two modes, both hipEvent pairs on the launch stream around each launch:
//  * kind (clipk_prof_enable): one kernel class, summed (total ms, launches, work);
//  * sites (clipk_prof_sites_enable): every named launch site of the encoders, with its
//    algorithmic FLOPs and HBM bytes, aggregated per site by clipk_prof_sites_read.
struct ProfState {
  int kind = CLIPK_PROF_NONE;
  bool sites = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  std::vector<double> work, bytes;
  std::vector<int> site;
  std::vector<const char*> names;  // site table (string literals)
  size_t used = 0;
};
static ProfState g_prof;

static int site_index(const char* name) {
  for (size_t i = 0; i < g_prof.names.size(); ++i)
    if (std::strcmp(g_prof.names[i], name) == 0) return (int)i;
  g_prof.names.push_back(name);
  return (int)g_prof.names.size() - 1;
}

struct ProfScope {
  bool on = false;
  hipStream_t st;
  size_t idx = 0;
  ProfScope(int cls, hipStream_t s, double work, const char* site = nullptr, double bytes = 0.0) : st(s) {
    bool take = false;
    if (g_prof.sites) {
      take = site != nullptr;
    } else if (g_prof.kind != CLIPK_PROF_NONE && cls != CLIPK_PROF_NONE) {
      const bool is_gemm = cls == CLIPK_PROF_GEMM_FC || cls == CLIPK_PROF_GEMM_ALL || cls == CLIPK_PROF_GEMM_DGELU;
      take = g_prof.kind == cls || (g_prof.kind == CLIPK_PROF_GEMM_ALL && is_gemm);
    }
    if (!take) return;
    if (g_prof.used == g_prof.ev.size()) {
      hipEvent_t a, b;
      if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
      g_prof.ev.push_back({a, b});
      g_prof.work.push_back(0.0);
      g_prof.bytes.push_back(0.0);
      g_prof.site.push_back(-1);
    }
    idx = g_prof.used++;
    g_prof.work[idx] = work;
    g_prof.bytes[idx] = bytes;
    g_prof.site[idx] = site ? site_index(site) : -1;
    on = hipEventRecord(g_prof.ev[idx].first, st) == hipSuccess;
  }
  ~ProfScope() {
    if (on) (void)hipEventRecord(g_prof.ev[idx].second, st);
  }
};

#define TRY(x)                 \
  do {                         \
    int _rc = (x);             \
    if (_rc != CLIPK_OK) return _rc; \
  } while (0)

// Algorithmic HBM bytes of one GEMM: A, B read once, out (+ out2) written, residual / aux
// read once (epi without the CLIPK_A_QGELU flag).
static double gemm_bytes(int in, int out, int epi, int M, int N, int K, bool has_o2, int auxdt) {
  const double a = esize(in), o = esize(out), wb = in == CLIPK_F32S16 ? 2.0 : a;  // compact weight
  double b = (double)M * K * a + (double)N * K * wb + (double)M * N * o * (has_o2 ? 2 : 1);
  const int e = epi & ~(CLIPK_A_QGELU | CLIPK_QGELU_DERIV | CLIPK_A_SPLIT | CLIPK_OUT_SPLIT | CLIPK_OUT2_SPLIT_GAMMA);
  if (e == CLIPK_EPI_BIAS_RES) b += (double)M * N * o;
  if (e == CLIPK_EPI_DQGELU) b += (double)M * N * esize(auxdt);
  return b;
}

// sk / skb: split-K workspace (vision: small M); nullptr = one launch over the tile grid
static int gemm(int in, int out, int epi, int M, int N, int K, const void* A, const void* B,
                const float* bias, const void* res, void* o, void* o2, const void* aux, int auxdt,
                hipStream_t st, int prof_cls, void* sk = nullptr, size_t skb = 0, const char* site = nullptr) {
  if (t_split && in == CLIPK_F32) in = t_split == 2 ? CLIPK_F32S16 : CLIPK_F32S;
  ProfScope ps(prof_cls, st, 2.0 * M * N * K, site,
               site ? gemm_bytes(in, out, epi, M, N, K, o2 != nullptr, auxdt) : 0.0);
  if (sk && (epi & ~CLIPK_QGELU_DERIV) != CLIPK_EPI_DQGELU)
    return clipk_gemm_splitk(in, out, epi, M, N, K, A, K, B, K, bias, res, N, o, N, o2, 0, sk, skb, st);
  return clipk_gemm(in, out, epi, M, N, K, A, K, B, K, bias, res, N, o, N, o2, aux, auxdt, N, st);
}

// split-K workspace for the block GEMMs of a vision forward at `rows` rows (0 when none splits)
static size_t vit_splitk_bytes(int act, int rows, int D) {
  const int shapes[4][2] = {{3 * D, D}, {D, D}, {4 * D, D}, {D, 4 * D}};  // (N, K)
  size_t best = 0;
  for (const auto& nk : shapes) {
    const size_t b = clipk_gemm_splitk_ws_bytes(rows, nk[0], clipk_gemm_auto_splits(act, rows, nk[0], nk[1]));
    best = b > best ? b : best;
  }
  return best;
}

// ---------------------------------------------------------------- text layout
struct TextBufs {
  // saved (per layer)
  // X / Xm: residual stream (layer inputs / post-attention), of the encoder's residual dtype
  std::vector<void*> X, Xm;
  std::vector<float*> mean1, rstd1, mean2, rstd2, lse;
  std::vector<void*> qkv, o, h;
  void* Xf = nullptr;  // final layer output (== X[layers])
  float *meanf = nullptr, *rstdf = nullptr;
  // forward temporaries (oc / xc: the last layer's attention output and residual input
  // gathered to the EOT rows, text_eot_last)
  void *xn = nullptr, *g = nullptr, *lnf = nullptr, *oc = nullptr, *xc = nullptr;
  // LN fold: per (row, 64-column group) statistics partials of the residual stream; mean /
  // rstd of the un-saved (inference) forward
  float *lnst = nullptr, *tm = nullptr, *tr = nullptr, *rnb = nullptr;
  size_t saved_bytes = 0, ws_bytes = 0;
};

// save=1: per-layer activations live in `saved`; save=0: buffers are reused across layers
// rd: residual dtype (-1: the text encoder's, res_dtype; the ViT's is fp32)
static TextBufs text_layout(const clipk_encoder* e, size_t rows, int nout, void* saved, void* ws, bool save,
                            int rd = -1) {
  TextBufs t;
  const size_t W = e->W, H = e->heads, a = esize(e->act), xs = esize(rd < 0 ? res_dtype(e) : rd);
  const int nl = e->layers;
  Carver sv(saved), wk(ws);
  Carver& S = save ? sv : wk;
  t.X.resize(nl + 1); t.Xm.resize(nl); t.mean1.resize(nl); t.rstd1.resize(nl);
  t.mean2.resize(nl); t.rstd2.resize(nl); t.lse.resize(nl); t.qkv.resize(nl); t.o.resize(nl);
  t.h.resize(nl);
  if (save) {
    for (int l = 0; l <= nl; ++l) t.X[l] = S.take(rows * W * xs);
    for (int l = 0; l < nl; ++l) {
      t.Xm[l] = S.take(rows * W * xs);
      t.mean1[l] = (float*)S.take(rows * 4); t.rstd1[l] = (float*)S.take(rows * 4);
      t.mean2[l] = (float*)S.take(rows * 4); t.rstd2[l] = (float*)S.take(rows * 4);
      t.lse[l] = (float*)S.take(rows * H * 4);
      t.qkv[l] = S.take(rows * 3 * W * a);
      t.o[l] = S.take(rows * W * a);
      t.h[l] = S.take(rows * 4 * W * a);
    }
    t.meanf = (float*)S.take((size_t)nout * 4);
    t.rstdf = (float*)S.take((size_t)nout * 4);
  } else {
    void* x0 = wk.take(rows * W * xs);
    void* x1 = wk.take(rows * W * xs);
    void* xm = wk.take(rows * W * xs);
    void* q = wk.take(rows * 3 * W * a);
    void* o = wk.take(rows * W * a);
    for (int l = 0; l <= nl; ++l) t.X[l] = (l & 1) ? x1 : x0;
    for (int l = 0; l < nl; ++l) {
      t.Xm[l] = xm; t.qkv[l] = q; t.o[l] = o; t.h[l] = nullptr;
      t.mean1[l] = t.rstd1[l] = t.mean2[l] = t.rstd2[l] = nullptr; t.lse[l] = nullptr;
    }
  }
  t.Xf = t.X[nl];
  t.xn = wk.take(rows * W * a);
  t.g = wk.take(rows * 4 * W * a);
  t.lnf = wk.take((size_t)nout * W * a);
  t.oc = wk.take((size_t)nout * W * a);
  t.xc = wk.take((size_t)nout * W * xs);
  t.lnst = (float*)wk.take(rows * (W / 64) * 8);
  t.tm = (float*)wk.take(rows * 4);
  t.tr = (float*)wk.take(rows * 4);
  t.rnb = (float*)wk.take(rows * 8);
  t.saved_bytes = save ? sv.off : 0;
  t.ws_bytes = wk.off;
  return t;
}

constexpr int kAmaxBlocks = 256;  // partial maxima of the fp32s gradient-scale reduction

struct TextBwdBufs {
  void *dtg, *dX_lp, *dh, *do_, *dqkv, *dxn;  // dxn: LN-output grads in the grad dtype
  float* dlnf;
  float* gscale;  // PREC fp32s: the backward's gradient scale s and 1 / s (+ amax partials)
  void* part;  // shared-prefix attention: per-chunk prefix dK/dV partials
  size_t bytes;
};

static TextBwdBufs text_bwd_layout(const clipk_encoder* e, size_t rows, int nout, size_t part_bytes,
                                   void* ws) {
  TextBwdBufs b;
  const size_t W = e->W, g = esize(e->grad);
  Carver c(ws);
  b.dtg = c.take((size_t)nout * e->E * g);
  b.dlnf = (float*)c.take((size_t)nout * W * 4);
  b.dX_lp = c.take(rows * W * g);
  b.dh = c.take(rows * 4 * W * g);
  b.dxn = c.take(rows * W * g);
  b.do_ = c.take(rows * W * g);
  b.dqkv = c.take(rows * 3 * W * g);
  b.part = part_bytes ? c.take(part_bytes) : nullptr;
  b.gscale = (float*)c.take((2 + kAmaxBlocks) * sizeof(float));
  b.bytes = c.off;
  return b;
}

// ---- PREC fp32s gradient scaling. The split-fp16 GEMMs keep ~22 bits of an operand only while
// its values sit in fp16's normal range (|x| >= 2^-2 for the lo part); gradients here are
// ~1e-4-sized. The text backward is linear in dtxt, so it runs on s * dtxt with s a power of
// two putting max |dtxt| in [64, 128) (1/512 of the fp16 maximum: headroom for growth through
// the layers), and the results are multiplied by 1 / s at the end -- both exact.
__global__ __launch_bounds__(256) void amax_partial_kernel(long n, const float* __restrict__ x,
                                                           float* __restrict__ part) {
  __shared__ float sm[4];
  float m = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) m = fmaxf(m, fabsf(x[i]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
}
// sc[0] = s, sc[1] = 1 / s from the partial maxima sc[2 ..]: m s in [2^(target-1), 2^target)
__global__ __launch_bounds__(64) void grad_scale_pick_kernel(int nparts, int target, float* __restrict__ sc) {
  float m = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 64) m = fmaxf(m, sc[2 + i]);
  m = wave_max(m);
  if (threadIdx.x == 0) {
    int ex = 0;
    if (m > 0.f && m < INFINITY) (void)frexpf(m, &ex);  // m = f 2^ex, f in [0.5, 1)
    const int k = min(max(target - ex, -120), 120);      // m * 2^k in [2^(target-1), 2^target)
    sc[0] = ldexpf(1.0f, k);
    sc[1] = ldexpf(1.0f, -k);
  }
}
__global__ __launch_bounds__(256) void scale_by_kernel(long n, const float* __restrict__ x, float* __restrict__ y,
                                                       const float* __restrict__ sc, int which) {
  const float s = sc[which];
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) y[i] = x[i] * s;
}
static int grad_scale_in(const clipk_encoder* e, long n, const float* x, float* y, float* sc, hipStream_t st) {
  hipLaunchKernelGGL(amax_partial_kernel, dim3(kAmaxBlocks), dim3(256), 0, st, n, x, sc + 2);
  hipLaunchKernelGGL(grad_scale_pick_kernel, dim3(1), dim3(64), 0, st, kAmaxBlocks, e->split_target, sc);
  hipLaunchKernelGGL(scale_by_kernel, dim3((unsigned)std::min<long>((n + 255) / 256, 4096)), dim3(256), 0, st, n, x, y,
                     (const float*)sc, 0);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}
static int grad_scale_out(long n, float* x, const float* sc, hipStream_t st) {
  hipLaunchKernelGGL(scale_by_kernel, dim3((unsigned)std::min<long>((n + 255) / 256, 8192)), dim3(256), 0, st, n, x, x,
                     sc, 1);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

// Overflow check of a split (PREC fp32s) call's results (clipk_encoder_set_status): status |= bit
// when any of nseg segments of seg_len floats (seg_stride apart) holds a non-finite value -- the
// fp16 parts of an operand past 65504 give inf, and inf - inf NaN, which reaches the outputs.
__global__ __launch_bounds__(256) void finite_check_kernel(int nseg, long seg_len, long seg_stride,
                                                           const float* __restrict__ x, int* __restrict__ status,
                                                           int bit) {
  const long n = (long)nseg * seg_len;
  bool bad = false;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    bad |= !__builtin_isfinite(x[(i / seg_len) * seg_stride + i % seg_len]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(status, bit);
}
static int split_check(const clipk_encoder* e, int nseg, long seg_len, long seg_stride, const float* x, int bit,
                       hipStream_t st) {
  if (!e->split || !e->status || nseg <= 0 || seg_len <= 0) return CLIPK_OK;
  const long nb = ((long)nseg * seg_len + 255) / 256;
  hipLaunchKernelGGL(finite_check_kernel, dim3((unsigned)std::min<long>(nb, 2048)), dim3(256), 0, st, nseg, seg_len,
                     seg_stride, x, e->status, bit);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

// Row structure of one encoder call: nseq plain sequences of length L (vision, unpacked
// text), or the shared-prefix packed text layout (attention_prefix.hip).
struct SeqShape {
  int rows = 0, nout = 0;
  int nseq = 0, L = 0, causal = 0;
  bool packed = false;
  int G = 0, C = 0, P = 0, R = 0, ntiles = 0;
  const int* tiles = nullptr;
  const int* row_first = nullptr;
  static SeqShape plain(int nseq, int L, int causal) {
    SeqShape s;
    s.rows = nseq * L; s.nout = nseq; s.nseq = nseq; s.L = L; s.causal = causal;
    return s;
  }
  static SeqShape prefix(int G, int C, int P, int R, int ntiles, const int* tiles, const int* row_first) {
    SeqShape s;
    s.rows = G * R; s.nout = G * C; s.packed = true; s.causal = 1;
    s.G = G; s.C = C; s.P = P; s.R = R; s.ntiles = ntiles; s.tiles = tiles; s.row_first = row_first;
    return s;
  }
  size_t part_bytes(int heads) const { return packed ? clipk_attention_prefix_ws_bytes(G, ntiles, heads) : 0; }
};

// pflags: clipk_attention_prefix_*_ex flags (CLIPK_PREFIX_CLS_GROUP0: layer 0 under forward sharing)
static int attn_fwd(const clipk_encoder* e, const SeqShape& sh, const void* qkv, void* o, float* lse,
                    hipStream_t st, int pflags = 0) {
  const int W = e->W;
  if (sh.packed)
    return clipk_attention_prefix_fwd_ex(e->act, sh.G, sh.P, sh.R, sh.ntiles, sh.tiles, sh.row_first, e->heads,
                                         qkv, 3 * W, o, W, lse, pflags, st);
  return clipk_attention_fwd(e->act, sh.nseq, sh.L, e->heads, sh.causal, qkv, 3 * W, o, W, lse, st);
}

// dqkv_split (shared-prefix packed rows, fp32 gradients): dq|dk|dv stored in the pre-split form the
// qkv input-grad GEMM reads with CLIPK_A_SPLIT (grad dtype CLIPK_F32S of the prefix backward)
static int attn_bwd(const clipk_encoder* e, const SeqShape& sh, const void* qkv, const void* o,
                    const void* dout, const float* lse, void* dqkv, void* part, hipStream_t st,
                    bool dqkv_split = false, int pflags = 0) {
  const int W = e->W;
  if (sh.packed)
    return clipk_attention_prefix_bwd_ex(e->act, dqkv_split ? CLIPK_F32S : e->grad, sh.G, sh.P, sh.R, sh.ntiles, sh.tiles, sh.row_first,
                                      e->heads, qkv, 3 * W, o, W, dout, W, lse, dqkv, 3 * W, part,
                                      sh.part_bytes(e->heads), pflags, st);
  return clipk_attention_bwd(e->act, e->grad, sh.nseq, sh.L, e->heads, sh.causal, qkv, 3 * W, o, W, dout, W,
                             lse, dqkv, 3 * W, st);
}

// Attention half of a residual block: xn = LN1(X); qkv = xn Win^T + b; o = attention(qkv).
static int block_attn(const clipk_encoder* e, const std::array<const void*, 16>& w, const SeqShape& sh, int rd,
                      const void* X, void* xn, void* qkv, void* o, float* lse, float* m1, float* r1,
                      hipStream_t st, bool text, void* sk, size_t skb) {
  const int pg = text ? CLIPK_PROF_GEMM_ALL : CLIPK_PROF_NONE;
  const int W = e->W, rows = sh.rows, act = e->act;
  const double lnb = (double)rows * W * (esize(rd) + esize(act)) + (m1 ? 8.0 * rows : 0.0);
  {
    ProfScope ps(CLIPK_PROF_NONE, st, 0.0, text ? "text.ln_fwd" : "vit.ln_fwd", lnb);
    TRY(clipk_layernorm_fwd_x(rd, act, rows, W, X, W, nullptr, (const float*)w[0], (const float*)w[1], xn, W,
                              m1, r1, st));
  }
  TRY(gemm(act, act, CLIPK_EPI_BIAS, rows, 3 * W, W, xn, w[2], (const float*)w[3], nullptr, qkv,
           nullptr, nullptr, 0, st, pg, sk, skb, text ? "text.qkv_fwd" : "vit.qkv_fwd"));
  {
    // algorithmic: read q|k|v, write o (+ the fp32 log-sum-exp when saved)
    const double ab = (double)rows * 4 * W * esize(act) + (lse ? 4.0 * rows * e->heads : 0.0);
    ProfScope ps(text ? CLIPK_PROF_ATTN : CLIPK_PROF_NONE, st, 0.0, text ? "text.attn_fwd" : "vit.attn_fwd", ab);
    TRY(attn_fwd(e, sh, qkv, o, lse, st));
  }
  return CLIPK_OK;
}

// Post-attention half over `rows` rows: Xm = X + o Wout^T + b; xn = LN2(Xm);
// Xo = Xm + MLP(xn). (The text encoder's last layer runs it on the EOT rows only.)
// Residual stream X, Xm, Xo of dtype rd (fp32, or the 16-bit act dtype for the text encoder).
// Training: c_fc writes both h (kept for the backward) and quickgelu(h) from its epilogue, and
// c_proj stages quickgelu(h) like any operand, so it runs the ping-pong loop. Knob
// CLIPK_TEXT_AQGELU=1: c_fc writes h alone and c_proj applies QuickGELU to A while staging it
// (register-staged 2-slot loop). Same-box A/B (profiles/r02o_ab_aqgelu.txt): 12.33 -> 12.19 ms
// per step with the epilogue form (c_proj 1.71 -> 1.22 ms, c_fc 1.19 -> 1.49 ms).
static bool a_qgelu_on() {
  static int v = -1;
  if (v < 0) {
    const char* s = getenv("CLIPK_TEXT_AQGELU");
    v = s ? atoi(s) : 0;
  }
  return v != 0;
}

// PREC fp32s: the MLP's hand-offs in pre-split form (include/clipk.h CLIPK_OUT_SPLIT / CLIPK_A_SPLIT):
// c_fc stores QuickGELU(h) as the fp16 parts c_proj's split would form, and the backward's dgelu
// stores dh as fc_dx's -- those GEMMs then run no split VALU in their K loop (23 % of their launch
// on the headline shapes, profiles/r06b/). Bitwise the same results. Knob CLIPK_PRESPLIT=0 (A/B).
static bool presplit_on() {
  static int v = -1;
  if (v < 0) {
    const char* s = getenv("CLIPK_PRESPLIT");
    v = s ? atoi(s) : 1;
  }
  return v != 0;
}
// the operand flags of one hand-off on this call's path (split encoder calls only)
static int ps_out() { return t_split && presplit_on() ? CLIPK_OUT_SPLIT : 0; }
static int ps_a() { return t_split && presplit_on() ? CLIPK_A_SPLIT : 0; }

// Training's c_fc saves quickgelu'(h) for the backward (CLIPK_QGELU_DERIV) instead of h itself;
// knob CLIPK_QGELU_DERIV=0 (A/B) saves h and the backward recomputes the derivative.
static bool qgelu_deriv_on() {
  static int v = -1;
  if (v < 0) {
    const char* s = getenv("CLIPK_QGELU_DERIV");
    v = s ? atoi(s) : 1;
  }
  return v != 0;
}

static int block_post(const clipk_encoder* e, const std::array<const void*, 16>& w, int rows, int rd,
                      const void* X, const void* o, void* Xm, void* Xo, void* xn, void* h, void* g, float* m2,
                      float* r2, hipStream_t st, bool text, void* sk, size_t skb) {
  const int pg = text ? CLIPK_PROF_GEMM_ALL : CLIPK_PROF_NONE;
  const int W = e->W, act = e->act;
  TRY(gemm(act, rd, CLIPK_EPI_BIAS_RES, rows, W, W, o, w[4], (const float*)w[5], X, Xm,
           nullptr, nullptr, 0, st, pg, sk, skb, text ? "text.out_fwd" : "vit.out_fwd"));
  {
    const double lnb = (double)rows * W * (esize(rd) + esize(act)) + (m2 ? 8.0 * rows : 0.0);
    ProfScope ps(CLIPK_PROF_NONE, st, 0.0, text ? "text.ln_fwd" : "vit.ln_fwd", lnb);
    TRY(clipk_layernorm_fwd_x(rd, act, rows, W, Xm, W, nullptr, (const float*)w[6], (const float*)w[7], xn, W,
                              m2, r2, st));
  }
  if (text && act != CLIPK_F32 && h && a_qgelu_on()) {
    // knob: c_fc writes only the pre-activation h and c_proj applies QuickGELU to its A
    // operand while staging it (no g write; measured slower than the ping-pong c_proj)
    TRY(gemm(act, act, CLIPK_EPI_BIAS, rows, 4 * W, W, xn, w[8], (const float*)w[9], nullptr, h,
             nullptr, nullptr, 0, st, CLIPK_PROF_GEMM_FC, nullptr, 0, "text.fc_fwd"));
    TRY(gemm(act, rd, CLIPK_EPI_BIAS_RES | CLIPK_A_QGELU, rows, W, 4 * W, h, w[10], (const float*)w[11], Xm,
             Xo, nullptr, nullptr, 0, st, pg, nullptr, 0, "text.proj_fwd"));
    return CLIPK_OK;
  }
  // training (h given): h receives quickgelu'(xn Wfc^T + b) for the backward (CLIPK_QGELU_DERIV)
  const int pso = sk ? 0 : ps_out(), psa = sk ? 0 : ps_a();  // (split-K slices take no pre-split operands)
  TRY(gemm(act, act, CLIPK_EPI_BIAS_QGELU | (h && qgelu_deriv_on() ? CLIPK_QGELU_DERIV : 0) | pso, rows, 4 * W, W, xn, w[8], (const float*)w[9],
           nullptr, g, h, nullptr, 0, st, text ? CLIPK_PROF_GEMM_FC : CLIPK_PROF_NONE, sk, skb, text ? "text.fc_fwd" : "vit.fc_fwd"));
  TRY(gemm(act, rd, CLIPK_EPI_BIAS_RES | psa, rows, W, 4 * W, g, w[10], (const float*)w[11], Xm, Xo,
           nullptr, nullptr, 0, st, pg, sk, skb, text ? "text.proj_fwd" : "vit.proj_fwd"));
  return CLIPK_OK;
}

// one residual block forward over all rows (shared by text and vision)
static int block_fwd(const clipk_encoder* e, const std::array<const void*, 16>& w, const SeqShape& sh,
                     int rd, const void* X, void* Xm, void* Xo, void* xn, void* qkv, void* o,
                     float* lse, void* h, void* g, float* m1, float* r1, float* m2, float* r2,
                     hipStream_t st, bool text, void* sk = nullptr, size_t skb = 0) {
  TRY(block_attn(e, w, sh, rd, X, xn, qkv, o, lse, m1, r1, st, text, sk, skb));
  return block_post(e, w, sh.rows, rd, X, o, Xm, Xo, xn, h, g, m2, r2, st, text, sk, skb);
}

// ---- LayerNorm fold (clipk_encoder_set_ln_fold; text encoder, 16-bit residual stream)
static int gemm_ln(int act, int epi, int M, int N, int K, const void* A, const void* B, const float* bias,
                   const void* res, void* o, void* o2, float* stats, const float* colsum, const float* rnb,
                   hipStream_t st, int prof_cls, const char* site, const float* gamma = nullptr) {
  const double b = gemm_bytes(act, act, epi, M, N, K, o2 != nullptr, act) + (stats ? (double)M * (N / 64) * 8 : 0.0) +
                   (rnb ? 8.0 * M : 0.0) + (gamma ? 4.0 * K : 0.0);
  ProfScope ps(prof_cls, st, 2.0 * M * N * K, site, b);
  // PREC fp32s: the split-packed weights. Split mode 2: every weight fp16-valued (CLIPK_F32S16),
  // the fold with gamma on A (B = W); mode 1 folds W' = W diag(gamma) into B (CLIPK_F32S)
  if (t_split && act == CLIPK_F32) act = t_split == 2 ? CLIPK_F32S16 : CLIPK_F32S;
  if (gamma) return clipk_gemm_ln_gamma(act, epi, M, N, K, A, K, B, K, bias, o, N, o2, colsum, rnb, gamma, st);
  return clipk_gemm_ln(act, epi, M, N, K, A, K, B, K, bias, res, N, o, N, o2, stats, colsum, rnb, st);
}
// PREC fp32s split mode 2 with pre-split hand-offs: the residual-stream producer (out_proj ->
// ln_2 -> c_fc, c_proj -> the next layer's ln_1 -> qkv) also stores the fold's A operand pre-split,
// split(x * gamma) (clipk_gemm_ln_stats_split), into xs; the fold reads it with CLIPK_A_SPLIT
static int gemm_ln_split2(int epi, int M, int N, int K, const void* A, const void* B, const float* bias,
                          const void* res, void* o, float* stats, const float* gamma, void* xs, hipStream_t st,
                          int prof_cls, const char* site) {
  const double b = gemm_bytes(CLIPK_F32S16, CLIPK_F32, epi, M, N, K, false, CLIPK_F32) + (double)M * (N / 64) * 8 +
                   4.0 * M * N + 4.0 * N;
  ProfScope ps(prof_cls, st, 2.0 * M * N * K, site, b);
  return clipk_gemm_ln_stats_split(CLIPK_F32S16, epi, M, N, K, A, K, B, K, bias, res, N, o, N, stats, gamma, xs, st);
}
// the fold-side hand-off of gemm_ln_split2 is on for this call: split mode 2, pre-split hand-offs
static bool ps_fold(const clipk_encoder* e) { return t_split == 2 && e->split == 2 && presplit_on(); }
// mean / rstd (kept for the LayerNorm backward) and the folding GEMM's (rstd, -rstd mean) pairs
static int ln_merge(int rows, int W, const float* lnst, float* m, float* r, float* rnb, hipStream_t st, bool text) {
  ProfScope ps(CLIPK_PROF_NONE, st, 0.0, text ? "text.ln_stats" : "vit.ln_stats", (double)rows * (W / 64) * 8 + 16.0 * rows);
  return clipk_ln_stats_merge(rows, W, lnst, m, r, rnb, st);
}
// the merge + fold pair as one clipk_gemm_ln_merge launch where the library runs it in-kernel
// (16-bit, the batch-1 text shapes), else the two launches under their own profiling sites
static int gemm_ln_merged(int act, int epi, int M, int N, int K, const void* A, const void* B, const float* bias,
                          void* o, void* o2, const float* lnst, const float* colsum, float* m, float* r,
                          float* rnb, hipStream_t st, int prof_cls, const char* site, bool text,
                          const float* gamma = nullptr) {
  if (t_split || act == CLIPK_F32 || !clipk_gemm_ln_merge_fused(act, M, N, K)) {
    TRY(ln_merge(M, K, lnst, m, r, rnb, st, text));
    return gemm_ln(act, epi, M, N, K, A, B, bias, nullptr, o, o2, nullptr, colsum, rnb, st, prof_cls, site, gamma);
  }
  const double b = gemm_bytes(act, act, epi, M, N, K, o2 != nullptr, act) + (double)M * (K / 64) * 8 + 16.0 * M;
  ProfScope ps(prof_cls, st, 2.0 * M * N * K, site, b);
  return clipk_gemm_ln_merge(act, epi, M, N, K, A, K, B, K, bias, o, N, o2, lnst, colsum, m, r, rnb, st);
}
// attention half: ln_1 statistics of X merged from the partials the previous layer's c_proj
// epilogue wrote (lnst); the qkv projection reads X itself through the fold
// (gamma: split mode 2, the fold's LayerNorm weight applied to A, f[0] = W itself)
static int block_attn_fold(const clipk_encoder* e, const std::array<const void*, 6>& f, const SeqShape& sh,
                           const void* X, void* qkv, void* o, float* lse, float* m1, float* r1, const float* lnst,
                           float* rnb, hipStream_t st, bool text, const float* gamma = nullptr,
                           const void* xs = nullptr) {
  // xs: split(X * gamma), written by the previous layer's c_proj (gemm_ln_split2): the fold's A
  const int W = e->W, rows = sh.rows, act = e->act;
  TRY(gemm_ln_merged(act, CLIPK_EPI_BIAS | (xs ? CLIPK_A_SPLIT : 0), rows, 3 * W, W, xs ? xs : X, f[0],
                     (const float*)f[2], qkv, nullptr, lnst, (const float*)f[1], m1, r1, rnb, st,
                     text ? CLIPK_PROF_GEMM_ALL : CLIPK_PROF_NONE, text ? "text.qkv_fwd" : "vit.qkv_fwd", text, gamma));
  const double ab = (double)rows * 4 * W * esize(act) + (lse ? 4.0 * rows * e->heads : 0.0);
  ProfScope ps(text ? CLIPK_PROF_ATTN : CLIPK_PROF_NONE, st, 0.0, text ? "text.attn_fwd" : "vit.attn_fwd", ab);
  return attn_fwd(e, sh, qkv, o, lse, st);
}
// post-attention half: out_proj writes Xm and its ln_2 statistics, c_fc reads Xm through the
// fold, c_proj writes Xo (and, when a next layer folds ln_1, its statistics)
static int block_post_fold(const clipk_encoder* e, const std::array<const void*, 16>& w,
                           const std::array<const void*, 6>& f, int rows, const void* X, const void* o, void* Xm,
                           void* Xo, void* h, void* g, float* m2, float* r2, float* lnst, float* rnb,
                           bool stats_next, hipStream_t st, bool text, void* xs = nullptr,
                           const float* gamma_next = nullptr) {
  // xs (split mode 2, pre-split hand-offs): scratch [rows, W] for split(Xm * gamma2) -- c_fc's A --
  // and then split(Xo * gamma_next), the next layer's qkv A (gamma_next: its ln_1 weight)
  const int W = e->W, act = e->act;
  const int pg = text ? CLIPK_PROF_GEMM_ALL : CLIPK_PROF_NONE;
  const float* g2 = e->split == 2 ? (const float*)w[6] : nullptr;
  if (xs)
    TRY(gemm_ln_split2(CLIPK_EPI_BIAS_RES, rows, W, W, o, w[4], (const float*)w[5], X, Xm, lnst, g2, xs, st, pg,
                       text ? "text.out_fwd" : "vit.out_fwd"));
  else
    TRY(gemm_ln(act, CLIPK_EPI_BIAS_RES, rows, W, W, o, w[4], (const float*)w[5], X, Xm, nullptr, lnst, nullptr,
                nullptr, st, pg, text ? "text.out_fwd" : "vit.out_fwd"));
  TRY(gemm_ln_merged(act, CLIPK_EPI_BIAS_QGELU | (h && qgelu_deriv_on() ? CLIPK_QGELU_DERIV : 0) | ps_out() |
                              (xs ? CLIPK_A_SPLIT : 0),
                     rows, 4 * W, W, xs ? xs : Xm, f[3], (const float*)f[5], g, h, lnst, (const float*)f[4], m2, r2,
                     rnb, st, text ? CLIPK_PROF_GEMM_FC : CLIPK_PROF_NONE, text ? "text.fc_fwd" : "vit.fc_fwd", text,
                     g2));
  if (stats_next && xs && gamma_next)
    return gemm_ln_split2(CLIPK_EPI_BIAS_RES | ps_a(), rows, W, 4 * W, g, w[10], (const float*)w[11], Xm, Xo, lnst,
                          gamma_next, xs, st, pg, text ? "text.proj_fwd" : "vit.proj_fwd");
  if (stats_next)
    return gemm_ln(act, CLIPK_EPI_BIAS_RES | ps_a(), rows, W, 4 * W, g, w[10], (const float*)w[11], Xm, Xo, nullptr,
                   lnst, nullptr, nullptr, st, pg, text ? "text.proj_fwd" : "vit.proj_fwd");
  return gemm(act, act, CLIPK_EPI_BIAS_RES | ps_a(), rows, W, 4 * W, g, w[10], (const float*)w[11], Xm, Xo, nullptr,
              nullptr, 0, st, pg, nullptr, 0, text ? "text.proj_fwd" : "vit.proj_fwd");
}

}  // namespace clipk

using namespace clipk;

extern "C" const char* clipk_strerror(int status) {
  switch (status) {
    case CLIPK_OK: return "ok";
    case CLIPK_EINVAL: return "invalid argument (null pointer or bad enum)";
    case CLIPK_ESHAPE: return "shape violates a kernel constraint";
    case CLIPK_EDTYPE: return "unsupported dtype combination";
    case CLIPK_EWORKSPACE: return "workspace too small";
    case CLIPK_ERANGE: return "input outside the supported range (clipk_split_pack: |W| >= 65504 / 64 or not finite; clipk_split_hi16: W not fp16-valued)";
    case CLIPK_EHIP: return "a HIP runtime call of a synchronous check failed";
    default: return status > 0 ? hipGetErrorString((hipError_t)status) : "unknown error";
  }
}

extern "C" int clipk_device_arch_ok(void) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 0;
  return std::strncmp(p.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

extern "C" int clipk_encoder_create(int width, int layers, int heads, int embed, int act_dtype,
                                    int grad_dtype, const void* const* layer_ptrs,
                                    const void* const* head_ptrs, clipk_encoder** out) {
  if (!layer_ptrs || !head_ptrs || !out) return CLIPK_EINVAL;
  if (width <= 0 || width % 128 || layers <= 0 || heads * 64 != width || embed % 128 || embed <= 0)
    return CLIPK_ESHAPE;
  if (act_dtype < 0 || act_dtype > 2 || grad_dtype < 0 || grad_dtype > 2) return CLIPK_EDTYPE;
  auto* e = new (std::nothrow) clipk_encoder();
  if (!e) return CLIPK_EINVAL;
  e->kind = 0; e->W = width; e->layers = layers; e->heads = heads; e->E = embed;
  e->act = act_dtype; e->grad = grad_dtype; e->res = e->patch = e->Kp = e->Limg = 0;
  e->lw.resize(layers);
  for (int l = 0; l < layers; ++l)
    for (int i = 0; i < 16; ++i) e->lw[l][i] = layer_ptrs[l * 16 + i];
  for (int i = 0; i < 4; ++i) e->head[i] = head_ptrs[i];
  for (int i = 4; i < 8; ++i) e->head[i] = nullptr;
  *out = e;
  return CLIPK_OK;
}

extern "C" int clipk_vision_create(int width, int layers, int heads, int embed, int res, int patch,
                                   int act_dtype, const void* const* layer_ptrs,
                                   const void* const* head_ptrs, clipk_encoder** out) {
  if (!layer_ptrs || !head_ptrs || !out) return CLIPK_EINVAL;
  if (width <= 0 || width % 128 || layers <= 0 || heads * 64 != width || embed % 128 || patch <= 0 ||
      res % patch)
    return CLIPK_ESHAPE;
  auto* e = new (std::nothrow) clipk_encoder();
  if (!e) return CLIPK_EINVAL;
  e->kind = 1; e->W = width; e->layers = layers; e->heads = heads; e->E = embed;
  e->act = act_dtype; e->grad = act_dtype; e->res = res; e->patch = patch;
  const int k = 3 * patch * patch;
  const int kq = act_dtype == CLIPK_F32 ? 32 : 64;
  e->Kp = (k + kq - 1) / kq * kq;
  e->Limg = (res / patch) * (res / patch) + 1;
  e->lw.resize(layers);
  for (int l = 0; l < layers; ++l)
    for (int i = 0; i < 16; ++i) e->lw[l][i] = layer_ptrs[l * 16 + i];
  for (int i = 0; i < 8; ++i) e->head[i] = head_ptrs[i];
  *out = e;
  return CLIPK_OK;
}

extern "C" void clipk_encoder_destroy(clipk_encoder* enc) { delete enc; }

namespace clipk {

// The text encoder's output is read at the EOT rows alone (ln_final + projection), so the
// last layer's out_proj, LN2 and MLP run on those nout rows only (C=1000 packed: 8,000 of
// 47,160 rows); its attention still covers every row, since the EOT rows attend to their
// whole prompt. Exact (all row-wise ops); knob CLIPK_TEXT_EOT_LAST=0 runs the full layer.
// Forward and backward must agree: the saved Xm / h / X[layers] of the last layer then hold
// nout compact rows.
static bool text_eot_last(const SeqShape& sh) {
  static int v = -1;
  if (v < 0) {
    const char* s = getenv("CLIPK_TEXT_EOT_LAST");
    v = s ? atoi(s) : 1;
  }
  return v != 0 && sh.nout < sh.rows;
}

// What differs between the text encoder and the ViT around the shared layer loop: residual
// dtype, final LayerNorm + projection (text: ln_final / text_projection on the EOT rows,
// model.py:606-616; ViT: ln_post / proj on the CLS rows, model.py:426-431), launch-site names.
struct EncIO {
  int rd;
  const float *lnf_w, *lnf_b;
  const void* proj_f;  // [E, W] act dtype (forward B operand)
  const void* proj_b;  // [W, E] grad dtype (backward B operand)
  bool text;
  void* sk = nullptr;  // split-K workspace for the forward GEMMs (ViT: small M)
  size_t skb = 0;
};
static EncIO text_io(const clipk_encoder* e) {
  EncIO io;
  io.rd = res_dtype(e);
  io.lnf_w = (const float*)e->head[0]; io.lnf_b = (const float*)e->head[1];
  io.proj_f = e->head[2]; io.proj_b = e->head[3];
  io.text = true;
  return io;
}
#define SITE(n) (io.text ? "text." n : "vit." n)

// LN fold in this call: set on the encoder, 16-bit residual stream (the text encoder's, or the
// ViT's forward, clipk_vit_forward) or PREC fp32s (fp32 stream, split GEMMs), no deep prompts (they rewrite rows between a producer's
// statistics and their use) and not the A-operand QuickGELU knob. Knob CLIPK_TEXT_LNFOLD=0 runs
// the LayerNorm passes.
static bool ln_fold_on(const clipk_encoder* e, const EncIO& io) {
  static int v = -1;
  if (v < 0) {
    const char* s = getenv("CLIPK_TEXT_LNFOLD");
    v = s ? atoi(s) : 1;
  }
  // clipk_ln_stats_merge covers widths that are multiples of 128 up to 1024; wider encoders run
  // the LayerNorm passes
  return v != 0 && (int)e->fold.size() == e->layers && (e->act != CLIPK_F32 || e->split) && io.rd == e->act &&
         e->W % 128 == 0 && e->W <= 1024 && !(e->deep.n_deep > 0 && e->deep.prompts) && !a_qgelu_on();
}

// deep prompts of layer l (1..n_deep) into the layer's input rows
static int deep_inject(const clipk_encoder* e, int l, int rd, void* X, hipStream_t st) {
  const DeepPrompts& d = e->deep;
  if (l < 1 || l > d.n_deep || !d.prompts) return CLIPK_OK;
  return clipk_rows_inject(rd, d.n_ctx, d.n_per, e->W, d.prompts + (size_t)(l - 1) * d.n_ctx * e->W, d.rows, X,
                           e->W, st);
}

// ---- prefix-input mode (clipk_encoder_set_input_rows), shared-prefix packed layout:
// * forward, layer 0, G >= 2: the class rows of every group enter layer 0 with the same values
//   (token embedding + position; CoCoOp's pi_b reaches only the context rows, all in the
//   prefix), and LN1 / the qkv projection are row-wise, so their q|k|v rows are computed once
//   (group 0) and copied to the other groups; the other groups' prefix rows are computed
//   compactly. Rows [0, R) of the LN1 statistics hold group 0's, rows [R, R + (G-1) P) the
//   other groups' prefix rows (layer 0's backward reads only prefix rows).
// * backward, layer 0: the encoder input's gradient is formed on the prefix rows only (its qkv
//   input-grad GEMM and LN1 backward run on G*P rows); other rows of dx0 are left unspecified.
// Exact: the same per-row arithmetic on the rows whose results are used.
static bool prefix_mode(const clipk_encoder* e, const SeqShape& sh) {
  return e->prefix_input && sh.packed && sh.P >= 1 && sh.R - sh.P >= sh.G * sh.P;
}
// prow[i] = g*R + p for prefix row i = g*P + p; with m/r: mc/rc[i] = the saved LN1 statistics of
// that row (at its own row, or -- forward sharing, `shared` -- at the layout described above)
__global__ __launch_bounds__(256) void prefix_tables_kernel(int G, int P, int R, int shared, int* __restrict__ prow,
                                                            const float* __restrict__ m, const float* __restrict__ r,
                                                            float* __restrict__ mc, float* __restrict__ rc) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= G * P) return;
  const int g = i / P, p = i % P;
  prow[i] = g * R + p;
  if (m) {
    const int si = (!shared || g == 0) ? g * R + p : R + (g - 1) * P + p;
    mc[i] = m[si];
    rc[i] = r[si];
  }
}
// rows [P, R) of group 0 (16-B chunks per row) copied to groups 1..G-1: each chunk read once
// and stored G-1 times
__global__ __launch_bounds__(256) void group_bcast_kernel(int G, int P, int R, int chunks, uint4* __restrict__ buf) {
  const long per = (long)(R - P) * chunks;
  for (long j = (long)blockIdx.x * 256 + threadIdx.x; j < per; j += (long)gridDim.x * 256) {
    const uint4 v = buf[(long)P * chunks + j];
    for (int g = 1; g < G; ++g) buf[(long)g * R * chunks + (long)P * chunks + j] = v;
  }
}
static int prefix_tables(const SeqShape& sh, bool shared, int* prow, const float* m, const float* r, float* mc,
                         float* rc, hipStream_t st) {
  const int n = sh.G * sh.P;
  hipLaunchKernelGGL(prefix_tables_kernel, dim3((n + 255) / 256), dim3(256), 0, st, sh.G, sh.P, sh.R, (int)shared, prow,
                     m, r, mc, rc);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

// Layer 0's attention half under forward sharing (prefix_mode, G >= 2): LN1 + qkv on group 0's
// rows and, compactly, on the other groups' prefix rows. The attention reads every group's class
// rows from group 0 (CLIPK_PREFIX_CLS_GROUP0), forward and backward: no per-group copies of them
// (127 MB per step at the 16-bit headline; 253 MB at fp32). Knob CLIPK_SHARE0_INDEX=0 copies them
// to every group (group_bcast_kernel) and reads them in place (A/B).
static bool share0_index_on() {
  static int v = -1;
  if (v < 0) {
    const char* s = getenv("CLIPK_SHARE0_INDEX");
    v = s ? atoi(s) : 1;
  }
  return v != 0;
}
static int block_attn_shared0(const clipk_encoder* e, const std::array<const void*, 16>& w, const SeqShape& sh,
                              int rd, const void* X, void* xn, void* qkv, void* o, float* lse, float* m1, float* r1,
                              int* prow, hipStream_t st) {
  const int W = e->W, act = e->act, G = sh.G, P = sh.P, R = sh.R;
  const int n = (G - 1) * P;  // other groups' prefix rows
  const size_t xa = (size_t)W * esize(act), qa = 3 * xa;
  TRY(prefix_tables(sh, true, prow, nullptr, nullptr, nullptr, nullptr, st));
  {
    ProfScope ps(CLIPK_PROF_NONE, st, 0.0, "text.ln_fwd", (double)(R + n) * W * (esize(rd) + esize(act)));
    TRY(clipk_layernorm_fwd_x(rd, act, R, W, X, W, nullptr, (const float*)w[0], (const float*)w[1], xn, W, m1, r1,
                              st));
    TRY(clipk_layernorm_fwd_x(rd, act, n, W, X, W, prow + P, (const float*)w[0], (const float*)w[1],
                              (char*)xn + (size_t)R * xa, W, m1 ? m1 + R : nullptr, r1 ? r1 + R : nullptr, st));
  }
  // one GEMM over [group 0's R rows | the compact prefix rows]: the compact rows land on rows
  // R.., of which group 1's prefix rows (R..R+P-1) are already in place
  TRY(gemm(act, act, CLIPK_EPI_BIAS, R + n, 3 * W, W, xn, w[2], (const float*)w[3], nullptr, qkv, nullptr, nullptr,
           0, st, CLIPK_PROF_GEMM_ALL, nullptr, 0, "text.qkv_fwd"));
  {
    ProfScope ps(CLIPK_PROF_NONE, st, 0.0, "text.qkv_bcast",
                 (double)(G - 2 > 0 ? G - 2 : 0) * P * qa * 2.0 + (share0_index_on() ? 0.0 : (double)(G - 1) * (R - P) * qa * 2.0));
    if (G > 2) TRY(clipk_rows_copy((int)qa, (G - 2) * P, (char*)qkv + (size_t)(R + P) * qa, nullptr, qkv, prow + 2 * P, st));
    if (!share0_index_on()) {
      const int chunks = (int)(qa / 16);
      const long total = (long)(R - P) * chunks;
      hipLaunchKernelGGL(group_bcast_kernel, dim3((unsigned)std::min<long>((total + 255) / 256, 4096)), dim3(256), 0,
                         st, G, P, R, chunks, (uint4*)qkv);
      CLIPK_CHECK_LAUNCH();
    }
  }
  {
    const double ab = (double)sh.rows * 4 * W * esize(act) + (lse ? 4.0 * sh.rows * e->heads : 0.0);
    ProfScope ps(CLIPK_PROF_ATTN, st, 0.0, "text.attn_fwd", ab);
    TRY(attn_fwd(e, sh, qkv, o, lse, st, share0_index_on() ? CLIPK_PREFIX_CLS_GROUP0 : 0));
  }
  return CLIPK_OK;
}

static int text_forward_impl(const clipk_encoder* e, const SeqShape& sh, const float* x0, const int* eot_rows,
                             float* txt, void* saved, size_t saved_bytes, void* ws, size_t ws_bytes,
                             hipStream_t st, const EncIO& io) {
  SplitScope split_scope(e);
  const bool save = saved != nullptr;
  TextBufs t = text_layout(e, sh.rows, sh.nout, saved, ws, save, io.rd);
  if (ws_bytes < t.ws_bytes || (save && saved_bytes < t.saved_bytes)) return CLIPK_EWORKSPACE;
  const int W = e->W, rows = sh.rows, rd = io.rd;
  const int pg = io.text ? CLIPK_PROF_GEMM_ALL : CLIPK_PROF_NONE;
  // layer-0 input: x0 (fp32) into X[0] (the residual dtype) when saving (LN1 backward reads
  // it) or when the residual stream is 16-bit
  const void* cur = x0;
  if (save || rd != CLIPK_F32) {
    if (rd == CLIPK_F32) {
      TRY(clipk_rows_copy(W * 4, rows, x0, nullptr, t.X[0], nullptr, st));  // (a clipk kernel, not a runtime blit)
    } else {
      TRY(clipk_cast(rd, (long)rows * W, x0, t.X[0], st));
    }
    cur = t.X[0];
  }
  const bool eotl = text_eot_last(sh);
  const int nl = e->layers, nout = sh.nout;
  const bool fold = ln_fold_on(e, io);
  bool have_stats = false;  // LN fold: t.lnst holds the statistics partials of cur
  bool xs_ready = false;    // t.xn holds split(cur * the next ln_1 weight) (block_post_fold)
  for (int l = 0; l < nl; ++l) {
    void* Xo = t.X[l + 1];
    if (!save && Xo == cur) Xo = t.X[l];  // ping-pong (cur may be the caller's x0)
    if (l >= 1) TRY(deep_inject(e, l, rd, const_cast<void*>(cur), st));  // l >= 1: cur is ours
    const bool share0 = l == 0 && io.text && sh.G >= 2 && prefix_mode(e, sh);
    // LN statistics of the un-saved forward go to temporaries (m1 is consumed before m2 is written)
    float* m1 = save ? t.mean1[l] : t.tm;
    float* r1 = save ? t.rstd1[l] : t.tr;
    float* m2 = save ? t.mean2[l] : t.tm;
    float* r2 = save ? t.rstd2[l] : t.tr;
    if (share0)
      TRY(block_attn_shared0(e, e->lw[l], sh, rd, cur, t.xn, t.qkv[l], t.o[l], t.lse[l], t.mean1[l], t.rstd1[l],
                             (int*)t.g, st));
    else if (fold && have_stats)
      TRY(block_attn_fold(e, e->fold[l], sh, cur, t.qkv[l], t.o[l], t.lse[l], m1, r1, t.lnst, t.rnb, st, io.text,
                          e->split == 2 ? (const float*)e->lw[l][0] : nullptr, xs_ready ? t.xn : nullptr));
    else
      TRY(block_attn(e, e->lw[l], sh, rd, cur, t.xn, t.qkv[l], t.o[l], t.lse[l], t.mean1[l], t.rstd1[l], st,
                     io.text, io.sk, io.skb));
    // post-attention half over every row, or -- last layer -- the EOT rows alone (the EOT rows
    // attend to their whole prefix, so the attention above covered every row); Xm, h, Xo then
    // hold nout compact rows
    const bool compact = eotl && l == nl - 1;
    const void* xin = cur;
    const void* oin = t.o[l];
    if (compact) {
      ProfScope ps(CLIPK_PROF_NONE, st, 0.0, SITE("eot_gather"), 2.0 * nout * W * (esize(e->act) + esize(rd)));
      TRY(clipk_rows_copy(W * (int)esize(e->act), nout, t.o[l], eot_rows, t.oc, nullptr, st));
      TRY(clipk_rows_copy(W * (int)esize(rd), nout, cur, eot_rows, t.xc, nullptr, st));
      xin = t.xc;
      oin = t.oc;
    }
    const int n = compact ? nout : sh.rows;
    // split mode 2, pre-split hand-offs: t.xn (free once layer 0's LayerNorm output is consumed)
    // carries split(x * gamma) from each residual producer to its fold
    void* xs = fold && ps_fold(e) ? t.xn : nullptr;
    const float* gnext = l + 1 < nl ? (const float*)e->lw[l + 1][0] : nullptr;
    xs_ready = xs && gnext;
    if (fold)
      TRY(block_post_fold(e, e->lw[l], e->fold[l], n, xin, oin, t.Xm[l], Xo, save ? t.h[l] : nullptr, t.g, m2, r2,
                          t.lnst, t.rnb, l + 1 < nl, st, io.text, xs, gnext));
    else
      TRY(block_post(e, e->lw[l], n, rd, xin, oin, t.Xm[l], Xo, t.xn, save ? t.h[l] : nullptr, t.g, t.mean2[l],
                     t.rstd2[l], st, io.text, compact ? nullptr : io.sk, compact ? 0 : io.skb));
    have_stats = fold && l + 1 < nl;
    cur = Xo;
  }
  // final LayerNorm on the output rows only (exact: LayerNorm is per row), then @ projection
  TRY(clipk_layernorm_fwd_x(rd, e->act, sh.nout, W, cur, W, eotl ? nullptr : eot_rows, io.lnf_w, io.lnf_b, t.lnf, W,
                            t.meanf, t.rstdf, st));
  TRY(gemm(e->act, CLIPK_F32, CLIPK_EPI_NONE, sh.nout, e->E, W, t.lnf, io.proj_f, nullptr, nullptr, txt,
           nullptr, nullptr, 0, st, pg, nullptr, 0, SITE("head")));
  return split_check(e, 1, (long)sh.nout * e->E, 0, txt, 1, st);
}

// Residual-gradient stream of the text backward: fp32, or the grad dtype when that is fp16
// (default: within the parity bar against the fp32 oracle, 1-cos(grad) <= 5e-5). The 16-bit
// stream is updated in place by each LayerNorm backward and is also the next GEMM's A
// operand, so the fp32 copy's 4 B/element read + write per LayerNorm disappear (LayerNorm
// backward 53 -> ~30 us per launch). CLIPK_TEXT_DRES16=0 keeps fp32, =1 also uses the
// stream for bf16 gradients.
static bool text_dres16(const clipk_encoder* e) {
  static int v = -2;
  if (v == -2) {
    const char* s = getenv("CLIPK_TEXT_DRES16");
    v = s ? atoi(s) : -1;
  }
  if (e->grad == CLIPK_F32 || v == 0) return false;
  return v > 0 || e->grad == CLIPK_F16;
}

// zero fill of 16-B aligned buffers of a multiple of 16 bytes (every text-backward buffer) as a
// clipk kernel instead of a runtime fill
__global__ __launch_bounds__(256) void zero16_kernel(long n, uint4* __restrict__ p) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = make_uint4(0, 0, 0, 0);
}
static int zero_bytes(void* p, size_t bytes, hipStream_t st) {
  if (bytes == 0) return CLIPK_OK;
  if ((bytes | (uintptr_t)p) & 15) return CLIPK_ESHAPE;
  const long n = (long)(bytes / 16);
  hipLaunchKernelGGL(zero16_kernel, dim3((unsigned)std::min<long>((n + 255) / 256, 4096)), dim3(256), 0, st, n,
                     (uint4*)p);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

static int text_backward_impl(const clipk_encoder* e, const SeqShape& sh, const int* eot_rows,
                              const float* dtxt, const void* saved, size_t saved_bytes, float* dx0,
                              void* ws, size_t ws_bytes, hipStream_t st, const EncIO& io) {
  SplitScope split_scope(e);
  TextBufs t = text_layout(e, sh.rows, sh.nout, const_cast<void*>(saved), nullptr, true, io.rd);
  TextBwdBufs b = text_bwd_layout(e, sh.rows, sh.nout, sh.part_bytes(e->heads), ws);
  if (saved_bytes < t.saved_bytes || ws_bytes < b.bytes) return CLIPK_EWORKSPACE;
  const int W = e->W, rows = sh.rows, nout = sh.nout, gd = e->grad, act = e->act;
  const int pg = io.text ? CLIPK_PROF_GEMM_ALL : CLIPK_PROF_NONE;
  float* dX = dx0;
  // d lnf = dtxt . P^T   (txt = lnf @ P, P = projection [W,E])
  if (e->split) {
    // PREC fp32s: the whole backward runs on s * dtxt (grad_scale_pick), unscaled at the end
    TRY(grad_scale_in(e, (long)nout * e->E, dtxt, (float*)b.dtg, b.gscale, st));
  } else {
    TRY(clipk_cast(gd, (long)nout * e->E, dtxt, b.dtg, st));
  }
  TRY(gemm(gd, CLIPK_F32, CLIPK_EPI_NONE, nout, W, e->E, b.dtg, io.proj_b, nullptr, nullptr, b.dlnf,
           nullptr, nullptr, 0, st, pg));
  // the ViT's residual stream is fp32: its gradient stays fp32 too
  const bool r16 = io.rd != CLIPK_F32 && text_dres16(e);
  // fp32 gradients with the fp32 stream (PREC fp32 / fp32s): the input-grad GEMMs read dX itself
  // (a second fp32 copy in dX_lp would be 4 B/element more per LayerNorm backward, unread).
  // PREC fp32s with pre-split hand-offs: the LayerNorm backwards also write dX_lp in the pre-split
  // form (lp dtype CLIPK_F32S), which proj_dx / out_dx read with CLIPK_A_SPLIT (no split VALU in
  // their K loops; +4 B/element written per LayerNorm backward)
  const bool a_split = e->split == 2 && presplit_on() && !r16 && gd == CLIPK_F32;  // (split mode 2: the kernels built)
  const bool lp_alias = !r16 && gd == CLIPK_F32 && !a_split;
  const int lpd = a_split ? CLIPK_F32S : gd;  // dX_lp's dtype
  const int dA_split = a_split ? CLIPK_A_SPLIT : 0;
  // ... and the shared-prefix attention backward writes dq|dk|dv pre-split for qkv_dx (+23 % on
  // that GEMM's launch when it splits them itself, as fc_dx before its pre-split A)
  // (knob CLIPK_PRESPLIT_QKV=0: qkv_dx splits them itself, A/B)
  static const bool qkv_knob = [] {
    const char* s = getenv("CLIPK_PRESPLIT_QKV");
    return s ? atoi(s) != 0 : true;
  }();
  const bool qkv_split = a_split && sh.packed && qkv_knob;
  const int dqkv_split = qkv_split ? CLIPK_A_SPLIT : 0;
  void* const dA = lp_alias ? (void*)dX : b.dX_lp;  // the A operand of proj_dx / out_dx
  const bool eotl = text_eot_last(sh);
  auto zero = [&](void* p, size_t bytes) { return zero_bytes(p, bytes, st); };
  if (!eotl) {
    // ln_final's gradient lands on the EOT rows of zeroed full-row streams
    if (!r16) TRY(zero(dX, (size_t)rows * W * 4));
    if (!lp_alias) TRY(zero(b.dX_lp, (size_t)rows * W * esize(gd)));
  }
  const int rd = io.rd;
  const int* frows = eotl ? nullptr : eot_rows;  // EOT-last: the last layer's rows are compact
  TRY(clipk_layernorm_bwd_x2(rd, CLIPK_F32, nout, W, b.dlnf, W, t.Xf, W, frows, io.lnf_w, t.meanf,
                             t.rstdf, nullptr, CLIPK_F32, W, r16 ? nullptr : dX, lp_alias ? nullptr : b.dX_lp, lpd,
                             frows, W, st));
  // residual-gradient update of one LayerNorm backward over n rows: dres (fp32 dX or the
  // 16-bit dX_lp, in place) + LN'(dxn); last: the encoder input's gradient, always fp32 into dX
  // algorithmic LN-backward bytes per row: dy (grad), x (residual dtype), residual gradient
  // read + written (16-bit stream or fp32), mean / rstd
  auto ln_bwd = [&](int n, const void* x, const float* gamma, const float* mean, const float* rstd, bool last) {
    const double lnbb = (double)n * W * (esize(gd) + esize(rd) + 2.0 * (r16 ? esize(gd) : 4)) + 8.0 * n;
    ProfScope ps(CLIPK_PROF_NONE, st, 0.0, SITE("ln_bwd"), lnbb);
    if (!r16)
      return clipk_layernorm_bwd_x(rd, gd, n, W, b.dxn, W, x, W, nullptr, gamma, mean, rstd, dX, W, dX,
                                   last || lp_alias ? nullptr : b.dX_lp, lpd, nullptr, W, st);
    return clipk_layernorm_bwd_x2(rd, gd, n, W, b.dxn, W, x, W, nullptr, gamma, mean, rstd, b.dX_lp, gd, W,
                                  last ? dX : nullptr, b.dX_lp, gd, nullptr, W, st);
  };
  // the forward saved quickgelu'(h) in t.h (CLIPK_QGELU_DERIV), except on the A-operand QuickGELU
  // knob's path (block_post), whose c_proj reads the pre-activation h itself
  const int dgelu_epi = (io.text && act != CLIPK_F32 && a_qgelu_on()) || !qgelu_deriv_on()
                            ? CLIPK_EPI_DQGELU
                            : (CLIPK_EPI_DQGELU | CLIPK_QGELU_DERIV);
  for (int l = e->layers - 1; l >= 0; --l) {
    const auto& w = e->lw[l];
    if (!w[12] || !w[13] || !w[14] || !w[15]) return CLIPK_EINVAL;
    const bool compact = eotl && l == e->layers - 1;
    const int n = compact ? nout : rows;  // rows of the post-attention half
    // MLP: dg = dX . Wproj ; dh = dg * qgelu'(h), qgelu'(h) saved by the forward's c_fc epilogue
    // in the act dtype (16-bit: rms 1.8e-4 on the derivative vs 2.9e-5 when recomputing it from a
    // 16-bit h -- under the 16-bit rounding of dh itself -- for no exp / rcp in this epilogue)
    // (the last layer's compact EOT-row launches are sites of their own: a different GEMM grid)
    // (PREC fp32s: dh handed to fc_dx pre-split, presplit_on; the saved-derivative form only)
    const bool dh_split = (dgelu_epi & CLIPK_QGELU_DERIV) != 0;
    TRY(gemm(gd, gd, dgelu_epi | (dh_split ? ps_out() | dA_split : 0), n, 4 * W, W, dA, w[15], nullptr, nullptr,
             b.dh, nullptr, t.h[l], act, st, io.text ? CLIPK_PROF_GEMM_DGELU : CLIPK_PROF_NONE, nullptr, 0,
             compact ? SITE("proj_dx_dgelu_eot") : SITE("proj_dx_dgelu")));
    TRY(gemm(gd, gd, CLIPK_EPI_NONE | (dh_split ? ps_a() : 0), n, W, 4 * W, b.dh, w[14], nullptr, nullptr, b.dxn,
             nullptr, nullptr, 0, st, pg, nullptr, 0, compact ? SITE("fc_dx_eot") : SITE("fc_dx")));
    TRY(ln_bwd(n, t.Xm[l], (const float*)w[6], t.mean2[l], t.rstd2[l], false));
    // attention: do = dXm . Wout ; dqkv ; dxn1 = dqkv . Win
    TRY(gemm(gd, gd, CLIPK_EPI_NONE | dA_split, n, W, W, dA, w[13], nullptr, nullptr, compact ? b.dh : b.do_,
             nullptr, nullptr, 0, st, pg, nullptr, 0, compact ? SITE("out_dx_eot") : SITE("out_dx")));
    if (compact) {
      // back to the full row layout: do and the residual gradient (the one LN1's backward
      // reads: the 16-bit stream, or fp32 dX) scattered to the EOT rows of zeroed buffers
      const int gb = W * (int)esize(gd), rb = W * (r16 ? (int)esize(gd) : 4);
      void* res = r16 ? b.dX_lp : (void*)dX;
      ProfScope ps(CLIPK_PROF_NONE, st, 0.0, SITE("eot_scatter"),
                   2.0 * nout * (gb + 2.0 * rb) + (double)rows * (gb + rb));
      TRY(zero(b.do_, (size_t)rows * gb));
      TRY(clipk_rows_copy(gb, nout, b.dh, nullptr, b.do_, eot_rows, st));
      TRY(clipk_rows_copy(rb, nout, res, nullptr, b.dqkv, nullptr, st));
      TRY(zero(res, (size_t)rows * rb));
      TRY(clipk_rows_copy(rb, nout, b.dqkv, nullptr, res, eot_rows, st));
    }
    {
      // algorithmic: read q|k|v (act), do (grad), lse; write dq|dk|dv (grad); the fp32 VALU
      // kernels also read o (the 16-bit MFMA ones recompute D_i = rowsum(P o dP) instead)
      const double ab = (double)rows * W * ((act == CLIPK_F32 ? 4.0 : 3.0) * esize(act) + 4.0 * esize(gd)) +
                        4.0 * rows * e->heads;
      ProfScope ps(io.text ? CLIPK_PROF_ATTN : CLIPK_PROF_NONE, st, 0.0, SITE("attn_bwd"), ab);
      // layer 0 under forward sharing: its class rows of q|k|v exist in group 0 only
      const bool shared0 = l == 0 && io.text && sh.G >= 2 && prefix_mode(e, sh) && share0_index_on();
      TRY(attn_bwd(e, sh, t.qkv[l], t.o[l], b.do_, t.lse[l], b.dqkv, b.part, st, qkv_split,
                   shared0 ? CLIPK_PREFIX_CLS_GROUP0 : 0));
    }
    if (l == 0 && io.text && prefix_mode(e, sh)) {
      // the input gradient on the prefix rows only: dqkv gathered to G*P compact rows, their
      // qkv input-grad GEMM and LN1 backward (scattered back to the prefix rows of dx0)
      const int np = sh.G * sh.P;
      int* prow = (int*)b.do_;  // do is free once the attention backward has run
      float* mc = (float*)(prow + np);
      float* rc = mc + np;
      TRY(prefix_tables(sh, sh.G >= 2, prow, t.mean1[0], t.rstd1[0], mc, rc, st));
      TRY(clipk_rows_copy(3 * W * (int)esize(gd), np, b.dqkv, prow, b.dh, nullptr, st));
      TRY(gemm(gd, gd, CLIPK_EPI_NONE | dqkv_split, np, W, 3 * W, b.dh, w[12], nullptr, nullptr, b.dxn, nullptr,
               nullptr, 0, st, pg, nullptr, 0, SITE("qkv_dx_prefix")));
      const float* g0 = (const float*)w[0];
      if (!r16)
        TRY(clipk_layernorm_bwd_x(rd, gd, np, W, b.dxn, W, t.X[0], W, prow, g0, mc, rc, dX, W, dX, nullptr, gd, prow,
                                  W, st));
      else
        TRY(clipk_layernorm_bwd_x2(rd, gd, np, W, b.dxn, W, t.X[0], W, prow, g0, mc, rc, b.dX_lp, gd, W, dX, b.dX_lp,
                                   gd, prow, W, st));
      continue;
    }
    TRY(gemm(gd, gd, CLIPK_EPI_NONE | dqkv_split, rows, W, 3 * W, b.dqkv, w[12], nullptr, nullptr, b.dxn,
             nullptr, nullptr, 0, st, pg, nullptr, 0, SITE("qkv_dx")));
    TRY(ln_bwd(rows, t.X[l], (const float*)w[0], t.mean1[l], t.rstd1[l], l == 0));
    const DeepPrompts& d = e->deep;
    if (l >= 1 && l <= d.n_deep && d.grads) {
      // layer l's replaced rows: their gradient is the prompt's; it stops there
      if (r16)
        TRY(clipk_rows_collect(gd, d.n_ctx, d.n_per, W, b.dX_lp, W, nullptr, 0, 0, d.rows,
                               d.grads + (size_t)(l - 1) * d.n_ctx * W, 0, 1, st));
      else
        TRY(clipk_rows_collect(CLIPK_F32, d.n_ctx, d.n_per, W, dX, W, lp_alias ? nullptr : b.dX_lp, gd, W, d.rows,
                               d.grads + (size_t)(l - 1) * d.n_ctx * W, 0, 1, st));
    }
  }
  if (e->split) {
    // undo the gradient scale (exact: a power of two) on everything this backward returned
    TRY(grad_scale_out((long)rows * W, dX, b.gscale, st));
    const DeepPrompts& d = e->deep;
    if (d.n_deep > 0 && d.grads) TRY(grad_scale_out((long)d.n_deep * d.n_ctx * W, d.grads, b.gscale, st));
    // the returned gradients must be finite (prefix-input mode: only the prefix rows of dx0 are
    // specified)
    if (io.text && prefix_mode(e, sh))
      TRY(split_check(e, sh.G, (long)sh.P * W, (long)sh.R * W, dX, 2, st));
    else
      TRY(split_check(e, 1, (long)rows * W, 0, dX, 2, st));
    if (d.n_deep > 0 && d.grads) TRY(split_check(e, 1, (long)d.n_deep * d.n_ctx * W, 0, d.grads, 2, st));
  }
  return CLIPK_OK;
}

static size_t text_ws_bytes(const clipk_encoder* e, size_t rows, int nout) {
  TextBufs a = text_layout(e, rows, nout, nullptr, nullptr, true);
  TextBufs b = text_layout(e, rows, nout, nullptr, nullptr, false);
  return a.ws_bytes > b.ws_bytes ? a.ws_bytes : b.ws_bytes;
}

}  // namespace clipk

extern "C" size_t clipk_text_saved_bytes(const clipk_encoder* e, int nseq, int L) {
  if (!e || nseq <= 0 || L <= 0) return 0;
  return text_layout(e, (size_t)nseq * L, nseq, nullptr, nullptr, true).saved_bytes;
}

extern "C" size_t clipk_text_ws_bytes(const clipk_encoder* e, int nseq, int L) {
  if (!e || nseq <= 0 || L <= 0) return 0;
  return text_ws_bytes(e, (size_t)nseq * L, nseq);
}

extern "C" int clipk_text_forward(const clipk_encoder* e, int nseq, int L, const float* x0,
                                  const int* eot_rows, float* txt, void* saved, size_t saved_bytes,
                                  void* ws, size_t ws_bytes, void* stream) {
  if (!e || e->kind != 0 || !x0 || !eot_rows || !txt || !ws) return CLIPK_EINVAL;
  if (nseq <= 0 || L <= 0 || L > 77) return CLIPK_ESHAPE;
  return text_forward_impl(e, SeqShape::plain(nseq, L, 1), x0, eot_rows, txt, saved, saved_bytes, ws,
                           ws_bytes, (hipStream_t)stream, text_io(e));
}

extern "C" size_t clipk_text_bwd_ws_bytes(const clipk_encoder* e, int nseq, int L) {
  if (!e || nseq <= 0 || L <= 0) return 0;
  return text_bwd_layout(e, (size_t)nseq * L, nseq, 0, nullptr).bytes;
}

extern "C" int clipk_text_backward(const clipk_encoder* e, int nseq, int L, const int* eot_rows,
                                   const float* dtxt, const void* saved, size_t saved_bytes, float* dx0,
                                   void* ws, size_t ws_bytes, void* stream) {
  if (!e || e->kind != 0 || !eot_rows || !dtxt || !saved || !dx0 || !ws) return CLIPK_EINVAL;
  if (!e->head[3]) return CLIPK_EINVAL;  // forward-only encoder
  if (nseq <= 0 || L <= 0 || L > 77) return CLIPK_ESHAPE;
  return text_backward_impl(e, SeqShape::plain(nseq, L, 1), eot_rows, dtxt, saved, saved_bytes, dx0, ws,
                            ws_bytes, (hipStream_t)stream, text_io(e));
}

static bool packed_ok(int G, int C, int P, int R, int ntiles) {
  return G > 0 && C > 0 && P >= 1 && P <= 16 && ntiles >= 1 && R >= P + C && (long)G * R < (1L << 31);
}

extern "C" size_t clipk_text_packed_saved_bytes(const clipk_encoder* e, int G, int C, int R) {
  if (!e || G <= 0 || C <= 0 || R <= 0) return 0;
  return text_layout(e, (size_t)G * R, G * C, nullptr, nullptr, true).saved_bytes;
}

extern "C" size_t clipk_text_packed_ws_bytes(const clipk_encoder* e, int G, int C, int R) {
  if (!e || G <= 0 || C <= 0 || R <= 0) return 0;
  return text_ws_bytes(e, (size_t)G * R, G * C);
}

extern "C" size_t clipk_text_packed_bwd_ws_bytes(const clipk_encoder* e, int G, int C, int R, int ntiles) {
  if (!e || G <= 0 || C <= 0 || R <= 0 || ntiles <= 0) return 0;
  return text_bwd_layout(e, (size_t)G * R, G * C, clipk_attention_prefix_ws_bytes(G, ntiles, e->heads), nullptr)
      .bytes;
}

extern "C" int clipk_text_forward_packed(const clipk_encoder* e, int G, int C, int P, int R, int ntiles,
                                         const int* tiles, const int* row_first, const float* x0,
                                         const int* eot_rows, float* txt, void* saved, size_t saved_bytes,
                                         void* ws, size_t ws_bytes, void* stream) {
  if (!e || e->kind != 0 || !tiles || !row_first || !x0 || !eot_rows || !txt || !ws) return CLIPK_EINVAL;
  if (!packed_ok(G, C, P, R, ntiles)) return CLIPK_ESHAPE;
  return text_forward_impl(e, SeqShape::prefix(G, C, P, R, ntiles, tiles, row_first), x0, eot_rows, txt, saved,
                           saved_bytes, ws, ws_bytes, (hipStream_t)stream, text_io(e));
}

extern "C" int clipk_text_backward_packed(const clipk_encoder* e, int G, int C, int P, int R, int ntiles,
                                          const int* tiles, const int* row_first, const int* eot_rows,
                                          const float* dtxt, const void* saved, size_t saved_bytes,
                                          float* dx0, void* ws, size_t ws_bytes, void* stream) {
  if (!e || e->kind != 0 || !tiles || !row_first || !eot_rows || !dtxt || !saved || !dx0 || !ws)
    return CLIPK_EINVAL;
  if (!e->head[3]) return CLIPK_EINVAL;
  if (!packed_ok(G, C, P, R, ntiles)) return CLIPK_ESHAPE;
  return text_backward_impl(e, SeqShape::prefix(G, C, P, R, ntiles, tiles, row_first), eot_rows, dtxt, saved,
                            saved_bytes, dx0, ws, ws_bytes, (hipStream_t)stream, text_io(e));
}

// ---------------------------------------------------------------- vision
namespace clipk {
struct VitBufs {
  void *patches, *xn, *qkv, *o, *g, *cls;
  float *pout, *x0, *x1, *xm;
  void* sk;  // split-K partials (small batches)
  size_t sk_bytes, bytes;
};
static VitBufs vit_layout(const clipk_encoder* e, int B, void* ws) {
  VitBufs v;
  const size_t a = esize(e->act), D = e->W, L = e->Limg, rows = (size_t)B * L;
  const size_t np = (size_t)B * (L - 1);
  Carver c(ws);
  v.patches = c.take(np * e->Kp * a);
  v.pout = (float*)c.take(np * D * 4);
  v.x0 = (float*)c.take(rows * D * 4);
  v.x1 = (float*)c.take(rows * D * 4);
  v.xm = (float*)c.take(rows * D * 4);
  v.xn = c.take(rows * D * a);
  v.qkv = c.take(rows * 3 * D * a);
  v.o = c.take(rows * D * a);
  v.g = c.take(rows * 4 * D * a);
  v.cls = c.take((size_t)B * D * a);
  // split-K (clipk_gemm_auto_splits) for the ViT GEMMs whose tile grid covers under half
  // of the CUs at small batch (the N = D projections); CLIPK_VIT_NOSPLITK turns it off
  static const bool no_sk = getenv("CLIPK_VIT_NOSPLITK") != nullptr;
  v.sk_bytes = no_sk ? 0 : vit_splitk_bytes(e->act, (int)rows, (int)D);
  v.sk = v.sk_bytes ? c.take(v.sk_bytes) : nullptr;
  v.bytes = c.off;
  return v;
}
}  // namespace clipk

namespace clipk {
static bool vit_res16(const clipk_encoder* e);
static size_t vit16_bytes(const clipk_encoder* e, int B, void* ws, void** parts);
static int vit16_forward(const clipk_encoder* e, int B, const float* img, float* feat, void* ws, size_t ws_bytes,
                         hipStream_t st);
}  // namespace clipk

extern "C" size_t clipk_vit_ws_bytes(const clipk_encoder* e, int B) {
  if (!e || e->kind != 1) return 0;
  if (vit_res16(e)) return vit16_bytes(e, B, nullptr, nullptr);
  return vit_layout(e, B, nullptr).bytes;
}

extern "C" int clipk_vit_forward(const clipk_encoder* e, int B, const float* img, float* feat,
                                 void* ws, size_t ws_bytes, void* stream) {
  if (!e || e->kind != 1 || !img || !feat || !ws) return CLIPK_EINVAL;
  if (B <= 0) return CLIPK_ESHAPE;
  if (vit_res16(e)) return vit16_forward(e, B, img, feat, ws, ws_bytes, (hipStream_t)stream);
  SplitScope split_scope(e);
  VitBufs v = vit_layout(e, B, ws);
  if (ws_bytes < v.bytes) return CLIPK_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int D = e->W, L = e->Limg, np = B * (L - 1), act = e->act;
  // head: 0 ln_pre_w 1 ln_pre_b 2 ln_post_w 3 ln_post_b 4 projT[E,D] 5 conv_w[D,Kp] 6 cls 7 pos
  TRY(clipk_im2col(act, B, e->res, e->patch, e->Kp, img, v.patches, st));
  TRY(gemm(act, CLIPK_F32, CLIPK_EPI_NONE, np, D, e->Kp, v.patches, e->head[5], nullptr, nullptr,
           v.pout, nullptr, nullptr, 0, st, CLIPK_PROF_NONE,
           clipk_gemm_splitk_ws_bytes(np, D, clipk_gemm_auto_splits(act, np, D, e->Kp)) <= v.sk_bytes ? v.sk : nullptr,
           v.sk_bytes, "vit.patch_embed"));
  TRY(clipk_vit_embed_ln(B, L, D, v.pout, (const float*)e->head[6], (const float*)e->head[7],
                         (const float*)e->head[0], (const float*)e->head[1], v.x0, st));
  float* cur = v.x0;
  float* nxt = v.x1;
  for (int l = 0; l < e->layers; ++l) {
    TRY(block_fwd(e, e->lw[l], SeqShape::plain(B, L, 0), CLIPK_F32, cur, v.xm, nxt, v.xn, v.qkv, v.o, nullptr, nullptr, v.g,
                  nullptr, nullptr, nullptr, nullptr, st, false, v.sk, v.sk_bytes));
    float* t = cur; cur = nxt; nxt = t;
  }
  // ln_post on the CLS rows (row stride L*D), then @ proj
  TRY(clipk_layernorm_fwd(act, B, D, cur, L * D, nullptr, (const float*)e->head[2],
                          (const float*)e->head[3], v.cls, D, nullptr, nullptr, st));
  TRY(gemm(act, CLIPK_F32, CLIPK_EPI_NONE, B, e->E, D, v.cls, e->head[4], nullptr, nullptr, feat,
           nullptr, nullptr, 0, st, CLIPK_PROF_NONE, nullptr, 0, "vit.head"));
  return split_check(e, 1, (long)B * e->E, 0, feat, 1, st);
}

// ---------------------------------------------------------------- prompted ViT (training)
// IVLP / MaPLe / PromptSRC (model.py:191-331, 401-431, 434-485): n_vpt visual prompt rows
// appended after the image tokens (rows per image L' = L + n_vpt), deep prompts replacing the
// last n_vpt rows at layers 1..n_deep (clipk_encoder_set_deep_prompts), and -- because those
// prompts train -- the input-grad backward of the whole ViT: the text encoder's layer loop
// (text_forward_impl / text_backward_impl) on plain non-causal rows with an fp32 residual
// stream, ln_post / proj on the CLS rows (the last layer's post-attention half on those rows
// only, as the text encoder's EOT rows).
namespace clipk {
static EncIO vit_io(const clipk_encoder* e, const void* proj_b) {
  EncIO io;
  io.rd = CLIPK_F32;
  io.lnf_w = (const float*)e->head[2]; io.lnf_b = (const float*)e->head[3];
  io.proj_f = e->head[4]; io.proj_b = proj_b;
  io.text = false;
  return io;
}
struct VitPBufs {
  void* patches;
  float *pout, *x0, *cls_rows;  // cls_rows: int row table [B] (as float storage, reinterpreted)
  float *dvpt_sum, *vmean, *vrstd;
  void* sk;
  size_t sk_bytes;
  void* rest;  // text_layout ws (forward) / text_bwd_layout (backward)
  size_t bytes;
};
static VitPBufs vitp_layout(const clipk_encoder* e, int B, int n_vpt, void* ws) {
  VitPBufs v;
  const size_t a = esize(e->act), D = e->W, L = e->Limg, Lp = L + n_vpt, rows = (size_t)B * Lp;
  const size_t np = (size_t)B * (L - 1);
  Carver c(ws);
  v.patches = c.take(np * e->Kp * a);
  v.pout = (float*)c.take(np * D * 4);
  v.x0 = (float*)c.take(rows * D * 4);
  v.cls_rows = (float*)c.take((size_t)B * 4);
  v.dvpt_sum = (float*)c.take((size_t)(n_vpt > 0 ? n_vpt : 1) * D * 4);
  v.vmean = (float*)c.take((size_t)(n_vpt > 0 ? n_vpt : 1) * 4);
  v.vrstd = (float*)c.take((size_t)(n_vpt > 0 ? n_vpt : 1) * 4);
  static const bool no_sk = getenv("CLIPK_VIT_NOSPLITK") != nullptr;
  v.sk_bytes = no_sk ? 0 : vit_splitk_bytes(e->act, (int)rows, (int)D);
  v.sk = v.sk_bytes ? c.take(v.sk_bytes) : nullptr;
  v.rest = ws ? (char*)ws + c.off : nullptr;
  const size_t fwd = text_layout(e, rows, B, nullptr, nullptr, true, CLIPK_F32).ws_bytes;
  const size_t fwd0 = text_layout(e, rows, B, nullptr, nullptr, false, CLIPK_F32).ws_bytes;
  const size_t bwd = text_bwd_layout(e, rows, B, 0, nullptr).bytes;
  v.bytes = c.off + std::max(std::max(fwd, fwd0), bwd);
  return v;
}
__global__ void cls_rows_kernel(int B, int Lp, int* rows) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) rows[b] = b * Lp;
}

// ---- ViT forward with a 16-bit residual stream (round 3; knob CLIPK_VIT_RES16=0 keeps fp32):
// the text encoder's layer loop (text_forward_impl) on B plain non-causal sequences, so the ViT
// gets the LayerNorm fold of ln_1 / ln_2 (when set on the handle) and the last layer's
// post-attention half on the CLS rows alone (the only rows ln_post reads; exact). ln_pre stays in
// clipk_vit_embed_ln (fp32 out, cast into the stream by the layer loop).
// Round 6: PREC fp32s (fp32 stream, split GEMMs) takes the same layer loop -- with the fp32
// residual stream, the LayerNorm fold (gamma on A in split mode 2) and its pre-split hand-offs,
// and the last layer's post-attention half on the CLS rows -- instead of block_fwd's LayerNorm
// passes over every row (knob CLIPK_VIT_LOOP32=0: the block_fwd form)
static bool vit_res16(const clipk_encoder* e) {
  static int v = -1, v32 = -1;
  if (v < 0) {
    const char* s = getenv("CLIPK_VIT_RES16");
    v = s ? atoi(s) : 1;
    const char* s32 = getenv("CLIPK_VIT_LOOP32");
    v32 = s32 ? atoi(s32) : 1;
  }
  if (e->act == CLIPK_F32) return v32 != 0 && e->split != 0;
  return v != 0;
}
// parts: patches, pout, x0, cls_rows, sk, rest (the layer loop's workspace); returns the bytes
static size_t vit16_bytes(const clipk_encoder* e, int B, void* ws, void** parts) {
  const size_t a = esize(e->act), D = e->W, L = e->Limg, rows = (size_t)B * L;
  const size_t np = (size_t)B * (L - 1);
  Carver c(ws);
  void* p[6];
  p[0] = c.take(np * e->Kp * a);
  p[1] = c.take(np * D * 4);
  p[2] = c.take(rows * D * 4);
  p[3] = c.take((size_t)B * 4);
  static const bool no_sk = getenv("CLIPK_VIT_NOSPLITK") != nullptr;
  const size_t skb = no_sk ? 0 : vit_splitk_bytes(e->act, (int)rows, (int)D);
  p[4] = skb ? c.take(skb) : nullptr;
  p[5] = ws ? (char*)ws + c.off : nullptr;
  if (parts)
    for (int i = 0; i < 6; ++i) parts[i] = p[i];
  return c.off + text_layout(e, rows, B, nullptr, nullptr, false, e->act).ws_bytes;
}
static int vit16_forward(const clipk_encoder* e, int B, const float* img, float* feat, void* ws, size_t ws_bytes,
                         hipStream_t st) {
  void* p[6];
  const size_t need = vit16_bytes(e, B, ws, p);
  if (ws_bytes < need) return CLIPK_EWORKSPACE;
  SplitScope split_scope(e);  // (PREC fp32s: the patch embedding's split GEMM, before the layer loop's own scope)
  const int D = e->W, L = e->Limg, np = B * (L - 1), act = e->act;
  const size_t skb = p[4] ? (size_t)((char*)p[5] - (char*)p[4]) : 0;
  TRY(clipk_im2col(act, B, e->res, e->patch, e->Kp, img, p[0], st));
  TRY(gemm(act, CLIPK_F32, CLIPK_EPI_NONE, np, D, e->Kp, p[0], e->head[5], nullptr, nullptr, p[1], nullptr, nullptr,
           0, st, CLIPK_PROF_NONE,
           clipk_gemm_splitk_ws_bytes(np, D, clipk_gemm_auto_splits(act, np, D, e->Kp)) <= skb ? p[4] : nullptr, skb,
           "vit.patch_embed"));
  TRY(clipk_vit_embed_ln(B, L, D, (const float*)p[1], (const float*)e->head[6], (const float*)e->head[7],
                         (const float*)e->head[0], (const float*)e->head[1], (float*)p[2], st));
  hipLaunchKernelGGL(cls_rows_kernel, dim3((B + 255) / 256), dim3(256), 0, st, B, L, (int*)p[3]);
  CLIPK_CHECK_LAUNCH();
  EncIO io = vit_io(e, nullptr);
  io.rd = act;
  io.sk = p[4];
  io.skb = skb;
  return text_forward_impl(e, SeqShape::plain(B, L, 0), (const float*)p[2], (const int*)p[3], feat, nullptr, 0, p[5],
                           need - (size_t)((char*)p[5] - (char*)ws), st, io);
}
// out[p] = sum over images b (fixed order) of dx[b * Lp + L + p]
__global__ __launch_bounds__(256) void vpt_rows_sum_kernel(int B, int Lp, int L, int n_vpt, int D,
                                                           const float* __restrict__ dx, float* __restrict__ out) {
  const int p = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (p >= n_vpt || c >= D) return;
  float acc = 0.f;
  for (int b = 0; b < B; ++b) acc += dx[((size_t)b * Lp + L + p) * D + c];
  out[(size_t)p * D + c] = acc;
}
}  // namespace clipk

extern "C" int clipk_encoder_set_input_rows(clipk_encoder* e, int mode) {
  if (!e) return CLIPK_EINVAL;
  if (mode != 0 && mode != 1) return CLIPK_EINVAL;
  e->prefix_input = mode;
  return CLIPK_OK;
}

extern "C" int clipk_encoder_set_ln_fold(clipk_encoder* e, const void* const* fold_ptrs) {
  if (!e) return CLIPK_EINVAL;
  if (!fold_ptrs) {
    e->fold.clear();
    return CLIPK_OK;
  }
  if (e->act == CLIPK_F32 && !e->split) return CLIPK_EDTYPE;  // fp32s: call after set_split
  std::vector<std::array<const void*, 6>> f(e->layers);
  for (int l = 0; l < e->layers; ++l)
    for (int i = 0; i < 6; ++i) {
      f[l][i] = fold_ptrs[l * 6 + i];
      if (!f[l][i]) return CLIPK_EINVAL;
    }
  e->fold.swap(f);
  return CLIPK_OK;
}

extern "C" int clipk_encoder_set_split(clipk_encoder* e, int on) {
  if (!e || on < 0 || on > 2) return CLIPK_EINVAL;
  if (on && (e->act != CLIPK_F32 || e->grad != CLIPK_F32)) return CLIPK_EDTYPE;
  // the mode names the weight tables' format (packed / compact) and what a fold table holds
  // (W diag(gamma) / W): fixed once set, and never changed under a fold
  if (on == e->split) return CLIPK_OK;
  if (e->split != 0 || !e->fold.empty()) return CLIPK_EINVAL;
  e->split = on;
  return CLIPK_OK;
}

extern "C" int clipk_encoder_set_split_target(clipk_encoder* e, int target) {
  if (!e || target < -24 || target > 30) return CLIPK_EINVAL;
  e->split_target = target;
  return CLIPK_OK;
}

extern "C" int clipk_encoder_set_status(clipk_encoder* e, int* status) {
  if (!e) return CLIPK_EINVAL;
  e->status = status;
  return CLIPK_OK;
}

extern "C" int clipk_encoder_set_deep_prompts(clipk_encoder* e, int n_deep, int n_ctx, int n_per, const int* rows,
                                              const float* prompts, float* grads) {
  if (!e) return CLIPK_EINVAL;
  if (n_deep < 0 || n_deep >= e->layers || (n_deep > 0 && (n_ctx <= 0 || n_per <= 0))) return CLIPK_ESHAPE;
  if (n_deep > 0 && (!rows || !prompts)) return CLIPK_EINVAL;
  e->deep = DeepPrompts();
  if (n_deep > 0) {
    e->deep.n_deep = n_deep; e->deep.n_ctx = n_ctx; e->deep.n_per = n_per;
    e->deep.rows = rows; e->deep.prompts = prompts; e->deep.grads = grads;
  }
  return CLIPK_OK;
}

extern "C" size_t clipk_vit_prompted_saved_bytes(const clipk_encoder* e, int B, int n_vpt) {
  if (!e || e->kind != 1 || B <= 0 || n_vpt < 0) return 0;
  return text_layout(e, (size_t)B * (e->Limg + n_vpt), B, nullptr, nullptr, true, CLIPK_F32).saved_bytes;
}

extern "C" size_t clipk_vit_prompted_ws_bytes(const clipk_encoder* e, int B, int n_vpt) {
  if (!e || e->kind != 1 || B <= 0 || n_vpt < 0) return 0;
  return vitp_layout(e, B, n_vpt, nullptr).bytes;
}

extern "C" int clipk_vit_forward_prompted(const clipk_encoder* e, int B, const float* img, int n_vpt,
                                          const float* vpt, float* feat, void* saved, size_t saved_bytes, void* ws,
                                          size_t ws_bytes, void* stream) {
  if (!e || e->kind != 1 || !img || !feat || !ws || (n_vpt > 0 && !vpt)) return CLIPK_EINVAL;
  if (B <= 0 || n_vpt < 0) return CLIPK_ESHAPE;
  SplitScope split_scope(e);
  VitPBufs v = vitp_layout(e, B, n_vpt, ws);
  if (ws_bytes < v.bytes) return CLIPK_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int D = e->W, L = e->Limg, Lp = L + n_vpt, np = B * (L - 1), act = e->act;
  TRY(clipk_im2col(act, B, e->res, e->patch, e->Kp, img, v.patches, st));
  TRY(gemm(act, CLIPK_F32, CLIPK_EPI_NONE, np, D, e->Kp, v.patches, e->head[5], nullptr, nullptr, v.pout, nullptr,
           nullptr, 0, st, CLIPK_PROF_NONE,
           clipk_gemm_splitk_ws_bytes(np, D, clipk_gemm_auto_splits(act, np, D, e->Kp)) <= v.sk_bytes ? v.sk : nullptr,
           v.sk_bytes, "vit.patch_embed"));
  TRY(clipk_vit_embed_ln_vpt(B, L, n_vpt, D, v.pout, (const float*)e->head[6], (const float*)e->head[7], vpt,
                             (const float*)e->head[0], (const float*)e->head[1], v.x0, st));
  hipLaunchKernelGGL(cls_rows_kernel, dim3((B + 63) / 64), dim3(64), 0, st, B, Lp, (int*)v.cls_rows);
  CLIPK_CHECK_LAUNCH();
  EncIO io = vit_io(e, nullptr);
  io.sk = v.sk; io.skb = v.sk_bytes;
  return text_forward_impl(e, SeqShape::plain(B, Lp, 0), v.x0, (const int*)v.cls_rows, feat, saved, saved_bytes,
                           v.rest, ws_bytes - ((char*)v.rest - (char*)ws), st, io);
}

extern "C" int clipk_vit_backward_prompted(const clipk_encoder* e, int B, int n_vpt, const float* vpt,
                                           const void* proj_bwd, const float* dfeat, const void* saved,
                                           size_t saved_bytes, float* dvpt, void* ws, size_t ws_bytes,
                                           void* stream) {
  if (!e || e->kind != 1 || !proj_bwd || !dfeat || !saved || !ws || (n_vpt > 0 && (!vpt || !dvpt)))
    return CLIPK_EINVAL;
  if (B <= 0 || n_vpt < 0) return CLIPK_ESHAPE;
  for (int l = 0; l < e->layers; ++l)
    if (!e->lw[l][12] || !e->lw[l][13] || !e->lw[l][14] || !e->lw[l][15]) return CLIPK_EINVAL;
  VitPBufs v = vitp_layout(e, B, n_vpt, ws);
  if (ws_bytes < v.bytes) return CLIPK_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int D = e->W, L = e->Limg, Lp = L + n_vpt;
  // the layer loop's gradient of the layer-0 input lands in x0's rows (fp32, [B*Lp, D])
  hipLaunchKernelGGL(cls_rows_kernel, dim3((B + 63) / 64), dim3(64), 0, st, B, Lp, (int*)v.cls_rows);
  CLIPK_CHECK_LAUNCH();
  TRY(text_backward_impl(e, SeqShape::plain(B, Lp, 0), (const int*)v.cls_rows, dfeat, saved, saved_bytes, v.x0,
                         v.rest, ws_bytes - ((char*)v.rest - (char*)ws), st, vit_io(e, proj_bwd)));
  if (n_vpt == 0) return CLIPK_OK;
  // first-layer prompts: x0 rows L.. of every image = ln_pre(vpt) (model.py:413-420); the
  // same vpt in every image, so d vpt = ln_pre'(vpt) . sum_b d x0[b, L + p] (linear in dy)
  TRY(clipk_layernorm_fwd(CLIPK_F32, n_vpt, D, vpt, D, nullptr, (const float*)e->head[0], (const float*)e->head[1],
                          v.dvpt_sum, D, v.vmean, v.vrstd, st));  // the statistics (output overwritten next)
  hipLaunchKernelGGL(vpt_rows_sum_kernel, dim3((D + 255) / 256, n_vpt), dim3(256), 0, st, B, Lp, L, n_vpt, D, v.x0,
                     v.dvpt_sum);
  CLIPK_CHECK_LAUNCH();
  return clipk_layernorm_bwd(CLIPK_F32, n_vpt, D, v.dvpt_sum, D, vpt, D, nullptr, (const float*)e->head[0], v.vmean,
                             v.vrstd, nullptr, D, dvpt, nullptr, CLIPK_F32, nullptr, D, st);
}

extern "C" int clipk_prof_enable(int kind) {
  g_prof.kind = kind;
  g_prof.sites = false;
  g_prof.used = 0;
  return CLIPK_OK;
}

extern "C" int clipk_prof_sites_enable(int on) {
  g_prof.sites = on != 0;
  g_prof.kind = CLIPK_PROF_NONE;
  g_prof.used = 0;
  return CLIPK_OK;
}

extern "C" int clipk_prof_sites_read(int max_sites, char* names, double* total_ms, long* count, double* flops,
                                     double* bytes, int* n_sites) {
  if (!n_sites || max_sites < 0 || (max_sites > 0 && (!names || !total_ms || !count || !flops || !bytes)))
    return CLIPK_EINVAL;
  const int ns = (int)g_prof.names.size();
  for (int i = 0; i < max_sites && i < ns; ++i) {
    std::strncpy(names + (size_t)i * CLIPK_PROF_NAME_LEN, g_prof.names[i], CLIPK_PROF_NAME_LEN - 1);
    names[(size_t)i * CLIPK_PROF_NAME_LEN + CLIPK_PROF_NAME_LEN - 1] = 0;
    total_ms[i] = 0.0; count[i] = 0; flops[i] = 0.0; bytes[i] = 0.0;
  }
  for (size_t i = 0; i < g_prof.used; ++i) {
    const int s = g_prof.site[i];
    if (s < 0 || s >= max_sites) continue;
    float ms = 0.f;
    if (hipEventSynchronize(g_prof.ev[i].second) != hipSuccess) return (int)hipGetLastError();
    if (hipEventElapsedTime(&ms, g_prof.ev[i].first, g_prof.ev[i].second) != hipSuccess)
      return (int)hipGetLastError();
    total_ms[s] += ms; count[s] += 1; flops[s] += g_prof.work[i]; bytes[s] += g_prof.bytes[i];
  }
  *n_sites = ns < max_sites ? ns : max_sites;
  g_prof.used = 0;
  return CLIPK_OK;
}

extern "C" int clipk_prof_read(double* total_ms, long* count, double* work) {
  double tot = 0.0, wsum = 0.0;
  for (size_t i = 0; i < g_prof.used; ++i) {
    float ms = 0.f;
    if (hipEventSynchronize(g_prof.ev[i].second) != hipSuccess) return (int)hipGetLastError();
    if (hipEventElapsedTime(&ms, g_prof.ev[i].first, g_prof.ev[i].second) != hipSuccess)
      return (int)hipGetLastError();
    tot += ms;
    wsum += g_prof.work[i];
  }
  if (total_ms) *total_ms = tot;
  if (count) *count = (long)g_prof.used;
  if (work) *work = wsum;
  g_prof.used = 0;
  return CLIPK_OK;
}
