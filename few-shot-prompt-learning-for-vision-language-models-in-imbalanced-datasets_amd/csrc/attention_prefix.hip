// Causal self-attention over SHARED-PREFIX packed prompts (the text encoder's hot layout).
//
// Under CLIP's causal text mask (PromptSRC/clip/model.py:592-598) the hidden state of token
// t depends only on tokens 0..t. CoCoOp's prompts for image b are
//     [SOT, ctx_1 + pi_b, ..., ctx_M + pi_b, class tokens, ".", EOT]
// (trainers/cocoop.py:173-198), so the first P = 1 + M rows are identical for all C
// classes of an image (CoOp: for all classes), and rows after a class's EOT never reach
// the EOT row that TextEncoder.forward reads (trainers/coop.py:201-203). The packed row
// layout therefore stores, per group g (one image, or the whole class set for CoOp),
//     [P prefix rows][class 0 rows P..eot_0][class 1 rows P..eot_1] ...
// (group stride R rows). Attention: the prefix rows attend among themselves (causal); a
// class row attends to all P prefix keys and causally to the rows of its own class.
// Exactly the reference's math, on ~ (P + sum q_len) / (C * L) of the rows.
//
// Work unit = a TILE of at most 16 consecutive class rows holding whole classes (the host
// packs consecutive classes greedily, so a 16-row MFMA tile carries ~16/q_len classes
// instead of one): tiles[2t], tiles[2t+1] = (group-relative first row, rows). row_first[r]
// = first row of the class that row r belongs to (the causal block-diagonal mask inside a
// tile). Unit 0 of every group is the prefix tile itself (keys = its own rows).
//
// One wave per (group, chunk of units, head): the prefix K/V of (g, h) are loaded once per
// wave and reused by every tile of the chunk. The backward accumulates the prefix rows'
// dK/dV over the chunk in registers and writes one fp32 partial per chunk;
// prefix_kv_reduce sums the chunks in a fixed order (deterministic).
#include <cstdlib>

#include "attn_common.h"

namespace clipk {

// tiles whose loads are issued together (template parameter; env CLIPK_PREFIX_*_BATCH)
constexpr int kValuChunkMin = 4;              // units per wave, fp32 kernels: at least (f32_uc)

// Units per wave of the MFMA kernels (env CLIPK_PREFIX_FWD_CHUNK / _BWD_CHUNK, read once).
static int chunk_env(const char* name, int def) {
  const char* e = getenv(name);
  const int v = e ? atoi(e) : def;
  return v >= 1 && v <= 16 ? v : def;
}
static int lds_slots();
// (the LDS-staged forward measured best at 4 units per wave, the register one at 8)
static int fwd_chunk() { static int c = chunk_env("CLIPK_PREFIX_FWD_CHUNK", lds_slots() ? 4 : 8); return c; }
static int bwd_chunk() { static int c = chunk_env("CLIPK_PREFIX_BWD_CHUNK", 16); return c; }
static int prefix_num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0, v = 0;
    n = (hipGetDevice(&dev) == hipSuccess &&
         hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            ? v
            : 256;
  }
  return n;
}
// Backward units per wave for this shape: bwd_chunk(), halved (down to 4) while the grid would
// give fewer than 8 waves per CU -- few groups (CoCoOp at 1 image per step, CoOp's single class
// set) otherwise leave most CUs idle (1 image: 240 waves of 16 units on 256 CUs).
static int bwd_uc(int G, int ntiles, int H) {
  int uc = bwd_chunk();
  while (uc > 4 && (long)G * H * ((ntiles + 1 + uc - 1) / uc) < 8L * prefix_num_cus()) uc /= 2;
  return uc;
}
// Units per wave of the fp32 kernels: the G * H * chunks waves sized to one round of `wpc`
// resident waves per CU (4..16 units). A fixed 8 gave the headline forward 3,840 waves for 3,072
// slots (1.25 rounds, the second a quarter full): forward 120 -> 101 us, backward 224 -> 208 us
// isolated (profiles/r04s/).
static int f32_uc(int G, int ntiles, int H, int wpc) {
  const long slots = (long)wpc * prefix_num_cus();
  const long uc = ((long)(ntiles + 1) * G * H + slots - 1) / slots;
  // at most 16: many groups (the eval's 100 images) keep several rounds of shorter waves
  return (int)(uc < kValuChunkMin ? kValuChunkMin : uc > 16 ? 16 : uc);
}
// resident waves per CU of the fp32 kernels at WPB = 2 (VGPRs: forward 146 -> 3 per SIMD,
// backward <= 256 -> 2; LDS: forward 24 KB, backward 34 KB per 2-wave block)
constexpr int kF32FwdWpc = 12, kF32BwdWpc = 8;
static int fwd_batch() { static int c = chunk_env("CLIPK_PREFIX_FWD_BATCH", 1); return c; }
static int bwd_batch() { static int c = chunk_env("CLIPK_PREFIX_BWD_BATCH", 2); return c; }
// Waves per block (4 or 8; env CLIPK_PREFIX_WPB). Waves are head-fastest, so 8 waves (H = 8)
// put all heads of a row range in one block: one CU reads whole qkv rows.
static int prefix_wpb() { static int c = chunk_env("CLIPK_PREFIX_WPB", 4) >= 8 ? 8 : 4; return c; }
static inline int n_chunks(int ntiles, int uc) { return (ntiles + 1 + uc - 1) / uc; }
// LDS-staged kernels (attn_prefix_*_lds): ring slots per wave (CLIPK_PREFIX_LDS: 0 = the
// register-operand kernels, 2 or 3) and waves per block (CLIPK_PREFIX_LDS_WPB: 1, 2 or 4).
// Bench shape (G 8, C 1000, P 5; clean-cache HIP events, tools/attn_sweep.py): backward
// 98.4 -> 82.4 us (0.50 -> 0.60 of HBM), forward 48.4 -> 43.0 us at 2 slots / 4 waves.
static int lds_slots() {
  static int c = -1;
  if (c < 0) {
    const char* e = getenv("CLIPK_PREFIX_LDS");
    c = e ? atoi(e) : 2;
    if (c != 0 && c != 2 && c != 3) c = 2;
  }
  return c;
}
static int lds_wpb() {
  static int c = -1;
  if (c < 0) {
    const char* e = getenv("CLIPK_PREFIX_LDS_WPB");
    c = e ? atoi(e) : 4;
    if (c != 1 && c != 2 && c != 4) c = 4;
  }
  return c;
}

// The chunk's tile table in one VGPR (lane i holds tiles[2*(u_begin-1) + i]), read back
// with v_readlane: no dependent scalar-memory round trip inside the tile loop.
__device__ __forceinline__ int load_tile_table(const int* __restrict__ tiles, int ntiles, int u_begin,
                                               int lane) {
  const int idx = 2 * (u_begin - 1) + lane;
  return (lane < 32 && idx >= 0 && idx < 2 * ntiles) ? tiles[idx] : 0;
}
__device__ __forceinline__ void tile_info(int tab, int P, int u, int u_begin, int& t0, int& n, int& pre) {
  if (u == 0) {
    t0 = 0; n = P; pre = 0;
  } else {
    const int i = 2 * (u - u_begin);
    t0 = __builtin_amdgcn_readlane(tab, i);
    n = min(__builtin_amdgcn_readlane(tab, i + 1), 16);
    pre = P;
  }
}

// Unconditional 16-B load: the caller clamps the row to a valid one (rows past the tile
// are masked out of P / dS, never zeroed): no exec-masked branch around the load, so the
// compiler counts the batch's loads (vmcnt(N)) instead of draining them.
__device__ __forceinline__ s16x8 ld16(const void* p) { return *reinterpret_cast<const s16x8*>(p); }
__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ------------------------------------------------------------------ forward, MFMA (16-bit)
struct TileRows {
  s16x8 q[2], k[2], v[2];
  int t0, n, pre, first;  // first: this lane's row's class start, tile-relative
};

template <typename T, int kFwdBatch, int WPB = 4>
__global__ __launch_bounds__(WPB * 64) void attn_prefix_fwd_mfma(int G, int P, int R, int ntiles,
                                                            const int* __restrict__ tiles,
                                                            const int* __restrict__ row_first, int H,
                                                            int nchunk, int uc, const T* __restrict__ qkv,
                                                            int ldq, T* __restrict__ out, int ldo,
                                                            float* __restrict__ lse, int cls0) {
  __shared__ CLIPK_LDS_ALIGN short sm[WPB][2][16 * TRS];  // per wave: prefix V, own V
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int wid = blockIdx.x * WPB + w;
  if (wid >= G * nchunk * H) return;  // wave-uniform; no block barriers below
  const int h = wid % H, k = (wid / H) % nchunk, g = wid / (H * nchunk);
  const int W = H * 64;
  short* sVp = sm[w][0];
  short* sVo = sm[w][1];
  const int gR = g * R;
  const T* qh = qkv + h * 64;

  const int u_begin = k * uc, u_end = min((k + 1) * uc, ntiles + 1);
  const int tab = load_tile_table(tiles, ntiles, u_begin, lane);
  auto load = [&](int u, TileRows& f) {
    tile_info(tab, P, u, u_begin, f.t0, f.n, f.pre);
    const int rl = f.t0 + min(r16, f.n - 1);
    const T* qp = qh + ((cls0 && u > 0 ? 0 : gR) + rl) * ldq;  // cls0: class rows read from group 0
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = 8 * g4 + 32 * kk;
      f.q[kk] = ld16(qp + c);
      f.k[kk] = ld16(qp + W + c);
      f.v[kk] = ld16(qp + 2 * W + c);
    }
    f.first = u == 0 ? 0 : row_first[rl] - f.t0;
  };

  const bool pok = r16 < P;
  const T* pp = qh + (gR + (pok ? r16 : 0)) * ldq;
  s16x8 kp[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int c = 8 * g4 + 32 * kk;
    kp[kk] = ld_row16(pp + W + c, pok);
    *reinterpret_cast<s16x8*>(sVp + r16 * TRS + c) = ld_row16(pp + 2 * W + c, pok);
  }
  auto body = [&](TileRows& cur) {
    const int n = cur.n, pre = cur.pre, first = cur.first;
    const bool qok = r16 < n;
    lds_fence();  // previous tile's transposed reads of sVo are done
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) *reinterpret_cast<s16x8*>(sVo + r16 * TRS + 8 * g4 + 32 * kk) = cur.v[kk];
    f32x4 sp = {0.f, 0.f, 0.f, 0.f}, so = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      sp = mfma32_t<T>(kp[kk], cur.q[kk], sp);     // sp[r] = S[query r16][prefix key 4g4+r]
      so = mfma32_t<T>(cur.k[kk], cur.q[kk], so);  // so[r] = S[query r16][own key 4g4+r]
    }
    float vp[4], vq[4], mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = 4 * g4 + r;
      vp[r] = key < pre ? sp[r] * kScale : -INFINITY;
      vq[r] = (key <= r16 && key >= first) ? so[r] * kScale : -INFINITY;  // key == r16 always valid
      mx = fmaxf(mx, fmaxf(vp[r], vq[r]));
    }
    mx = xmax4(mx);
    float ep[4], eo[4], ps = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ep[r] = __expf(vp[r] - mx);
      eo[r] = __expf(vq[r] - mx);
      ps += ep[r] + eo[r];
    }
    ps = xsum4(ps);
    lds_fence();
    // O^T = V^T P^T: the transposed V read doubles as the A operand (A[m=d][k=key]) and the
    // probabilities as B (B[k=key 4g4+jj][n=query r16]), so lane (r16, g4) ends up holding
    // O[query r16][d = 16t + 4g4 .. +3]: one 8-byte store per 16 columns.
    const s16x4 bp = pack4<T>(ep[0], ep[1], ep[2], ep[3]);
    const s16x4 bo = pack4<T>(eo[0], eo[1], eo[2], eo[3]);
    const float inv = 1.0f / ps;
    f32x4 o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      o[t] = mfma16_t<T>(tr_read(sVp, 4 * g4, 16 * t, lane), bp, (f32x4){0.f, 0.f, 0.f, 0.f});
      o[t] = mfma16_t<T>(tr_read(sVo, 4 * g4, 16 * t, lane), bo, o[t]);
    }
    store_tile64<T>(out + (gR + cur.t0 + r16) * ldo + h * 64, o, inv, qok);
    if (lse && g4 == 0 && qok) lse[(gR + cur.t0 + r16) * H + h] = mx + __logf(ps);
  };
  // Batches of tiles: all their loads issued up front (unconditional, clamped), then the
  // bodies; waits are counted inside one loop iteration (a load carried across the back
  // edge gets a vmcnt(0) at the loop head).
  for (int u = u_begin; u < u_end; u += kFwdBatch) {
    TileRows rr[kFwdBatch];
#pragma unroll
    for (int j = 0; j < kFwdBatch; ++j) load(min(u + j, u_end - 1), rr[j]);
    __builtin_amdgcn_sched_barrier(0);  // every load of the batch issues before the first wait
#pragma unroll
    for (int j = 0; j < kFwdBatch; ++j)
      if (u + j < u_end) body(rr[j]);
  }
}

// ------------------------------------------------------------------ backward, MFMA (math in the grad dtype)
// Per tile, with the two 16-key tiles (prefix, own) handled like attn_bwd_mfma16: S / dP in
// both accumulator layouts, D_i = rowsum(P o dP) over both key tiles in registers; then the
// transposed products (operands swapped) dV^T = dO^T P, dK^T = Q^T dS, dQ^T = K^T dS^T so
// that each lane holds 4 consecutive columns of one row for the stores.
struct TileRowsB {
  s16x8 q[2], k[2], v[2], d[2];
  float l2, l1[4];
  int t0, n, pre, first2, first1[4];  // class starts (tile-relative) of rows r16 and 4g4+r
};

template <typename T, typename TG, int kBwdBatch, int WPB = 4>
__global__ __launch_bounds__(WPB * 64) void attn_prefix_bwd_mfma(int G, int P, int R, int ntiles,
                                                            const int* __restrict__ tiles,
                                                            const int* __restrict__ row_first, int H,
                                                            int nchunk, int uc, const T* __restrict__ qkv,
                                                            int ldq, const TG* __restrict__ dout,
                                                            int lddo, const float* __restrict__ lse,
                                                            TG* __restrict__ dqkv, int lddq,
                                                            float* __restrict__ part, int cls0) {
  static_assert(sizeof(T) == 2 && sizeof(TG) == 2, "MFMA attention backward: 16-bit operands, math in TG");
  __shared__ CLIPK_LDS_ALIGN short sm[WPB][4][16 * TRS];  // per wave: K_pre, K_own, Q, dO
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int wid = blockIdx.x * WPB + w;
  if (wid >= G * nchunk * H) return;  // wave-uniform
  const int h = wid % H, k = (wid / H) % nchunk, g = wid / (H * nchunk);
  const int W = H * 64;
  short* tKp = sm[w][0];
  short* tKo = sm[w][1];
  short* tQ = sm[w][2];
  short* tD = sm[w][3];
  const int gR = g * R;
  const T* qh = qkv + h * 64;
  const TG* dh = dout + h * 64;
  const float* lse_h = lse + h;

  const int u_begin = k * uc, u_end = min((k + 1) * uc, ntiles + 1);
  const int tab = load_tile_table(tiles, ntiles, u_begin, lane);
  auto load = [&](int u, TileRowsB& f) {
    tile_info(tab, P, u, u_begin, f.t0, f.n, f.pre);
    const int rl = f.t0 + min(r16, f.n - 1);
    const T* qp = qh + ((cls0 && u > 0 ? 0 : gR) + rl) * ldq;  // cls0: class rows read from group 0
    const TG* dp = dh + (gR + rl) * lddo;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = 8 * g4 + 32 * kk;
      f.q[kk] = ld16(qp + c);
      f.k[kk] = ld16(qp + W + c);
      f.v[kk] = ld16(qp + 2 * W + c);
      f.d[kk] = ld16(dp + c);
    }
    f.l2 = lse_h[(gR + rl) * H];
    f.first2 = u == 0 ? 0 : row_first[rl] - f.t0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ri = f.t0 + min(4 * g4 + r, f.n - 1);
      f.l1[r] = lse_h[(gR + ri) * H];
      f.first1[r] = u == 0 ? 0 : row_first[ri] - f.t0;
    }
  };

  const bool pok = r16 < P;
  const T* pp = qh + (gR + (pok ? r16 : 0)) * ldq;
  s16x8 kp[2], vp[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int c = 8 * g4 + 32 * kk;
    kp[kk] = to_g8<T, TG>(ld_row16(pp + W + c, pok));
    vp[kk] = to_g8<T, TG>(ld_row16(pp + 2 * W + c, pok));
    *reinterpret_cast<s16x8*>(tKp + r16 * TRS + c) = kp[kk];
  }
  f32x4 dkp[4], dvp[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    dkp[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    dvp[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  auto body = [&](TileRowsB& cur, bool own_is_prefix) {
    const int n = cur.n, pre = cur.pre;
    const bool qok = r16 < n;
    s16x8 q[2], ko[2], vo[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      q[kk] = to_g8<T, TG>(cur.q[kk]);
      ko[kk] = to_g8<T, TG>(cur.k[kk]);
      vo[kk] = to_g8<T, TG>(cur.v[kk]);
    }
    const s16x8* d = cur.d;
    lds_fence();  // previous tile's transposed reads are done
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = 8 * g4 + 32 * kk;
      *reinterpret_cast<s16x8*>(tQ + r16 * TRS + c) = q[kk];
      *reinterpret_cast<s16x8*>(tKo + r16 * TRS + c) = ko[kk];
      *reinterpret_cast<s16x8*>(tD + r16 * TRS + c) = d[kk];
    }
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    f32x4 s1p = z, s2p = z, p1p = z, p2p = z, s1o = z, s2o = z, p1o = z, p2o = z;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      s1p = mfma32_t<TG>(q[kk], kp[kk], s1p);   // S  [i=4g4+r][j=r16]
      s2p = mfma32_t<TG>(kp[kk], q[kk], s2p);   // S^T[j=4g4+r][i=r16]
      p1p = mfma32_t<TG>(d[kk], vp[kk], p1p);   // dP [i][j]
      p2p = mfma32_t<TG>(vp[kk], d[kk], p2p);   // dP^T
      s1o = mfma32_t<TG>(q[kk], ko[kk], s1o);
      s2o = mfma32_t<TG>(ko[kk], q[kk], s2o);
      p1o = mfma32_t<TG>(d[kk], vo[kk], p1o);
      p2o = mfma32_t<TG>(vo[kk], d[kk], p2o);
    }
    // layout 2: i = r16, j = 4g4+r  (rows past the tile are clamped copies: masked, not zeroed)
    float P2p[4], P2o[4], Dsum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 4 * g4 + r;
      P2p[r] = (qok && j < pre) ? __expf(s2p[r] * kScale - cur.l2) : 0.f;
      P2o[r] = (qok && j <= r16 && j >= cur.first2) ? __expf(s2o[r] * kScale - cur.l2) : 0.f;
      Dsum += P2p[r] * p2p[r] + P2o[r] * p2o[r];
    }
    Dsum = xsum4(Dsum);  // D_i for i = r16
    float dS2p[4], dS2o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dS2p[r] = P2p[r] * (p2p[r] - Dsum);
      dS2o[r] = P2o[r] * (p2o[r] - Dsum);
    }
    // layout 1: i = 4g4+r, j = r16
    float P1p[4], P1o[4], dS1p[4], dS1o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * g4 + r;
      const bool iok = i < n;
      const float Di = __shfl(Dsum, i, 64);
      P1p[r] = (iok && r16 < pre) ? __expf(s1p[r] * kScale - cur.l1[r]) : 0.f;
      P1o[r] = (iok && r16 <= i && r16 >= cur.first1[r]) ? __expf(s1o[r] * kScale - cur.l1[r]) : 0.f;
      dS1p[r] = P1p[r] * (p1p[r] - Di);
      dS1o[r] = P1o[r] * (p1o[r] - Di);
    }
    const s16x4 bPp = pack4<TG>(P1p[0], P1p[1], P1p[2], P1p[3]);      // B[k=i][n=j]
    const s16x4 bSp = pack4<TG>(dS1p[0], dS1p[1], dS1p[2], dS1p[3]);
    const s16x4 bPo = pack4<TG>(P1o[0], P1o[1], P1o[2], P1o[3]);
    const s16x4 bSo = pack4<TG>(dS1o[0], dS1o[1], dS1o[2], dS1o[3]);
    const s16x4 bTp = pack4<TG>(dS2p[0], dS2p[1], dS2p[2], dS2p[3]);  // B[k=j][n=i]
    const s16x4 bTo = pack4<TG>(dS2o[0], dS2o[1], dS2o[2], dS2o[3]);
    lds_fence();
    // one output (16 rows x 64) at a time, so only one 16-register tile is live for the
    // widened store
    TG* orow = dqkv + (gR + cur.t0 + r16) * lddq + h * 64;
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[t] = mfma16_t<TG>(tr_read(tKp, 4 * g4, 16 * t, lane), bTp, z);
      acc[t] = mfma16_t<TG>(tr_read(tKo, 4 * g4, 16 * t, lane), bTo, acc[t]);
    }
    store_tile64<TG>(orow, acc, kScale, qok);  // dQ
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const s16x4 aQ = tr_read(tQ, 4 * g4, 16 * t, lane);
      dkp[t] = mfma16_t<TG>(aQ, bSp, dkp[t]);
      acc[t] = mfma16_t<TG>(aQ, bSo, z);
      if (own_is_prefix) dkp[t] += acc[t];  // the prefix tile's keys are the prefix rows themselves
    }
    if (!own_is_prefix) store_tile64<TG>(orow + W, acc, kScale, qok);  // dK (wave-uniform branch)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const s16x4 aD = tr_read(tD, 4 * g4, 16 * t, lane);
      dvp[t] = mfma16_t<TG>(aD, bPp, dvp[t]);
      acc[t] = mfma16_t<TG>(aD, bPo, z);
      if (own_is_prefix) dvp[t] += acc[t];
    }
    if (!own_is_prefix) store_tile64<TG>(orow + 2 * W, acc, 1.0f, qok);  // dV
  };
  for (int u = u_begin; u < u_end; u += kBwdBatch) {
    TileRowsB rr[kBwdBatch];
#pragma unroll
    for (int j = 0; j < kBwdBatch; ++j) load(min(u + j, u_end - 1), rr[j]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < kBwdBatch; ++j)
      if (u + j < u_end) body(rr[j], u + j == 0);
  }
  // this chunk's partial dK/dV of the prefix rows (fp32, [G][nchunk][16][2W])
  float* pb = part + ((size_t)g * nchunk + k) * 16 * (2 * W);
  if (r16 < P) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float* dst = pb + (size_t)r16 * 2 * W + h * 64 + 16 * t + 4 * g4;
      *reinterpret_cast<f32x4*>(dst) = dkp[t] * kScale;
      *reinterpret_cast<f32x4*>(dst + W) = dvp[t];
    }
  }
}

// ------------------------------------------------------------------ LDS-staged MFMA kernels
// The kernels above load each lane's operand fragment straight into registers: one load
// instruction covers 16 rows x 64 B (half of each 128-B head slice), and a wave waits out a
// full load latency per batch of tiles. Here a tile's head slices arrive by global_load_lds
// (16 B per lane, lane-linear: one instruction = 8 whole 128-B rows) into a per-wave LDS ring
// of NS slots, NS-1 tiles ahead of the one being computed, so the next tiles' bytes are in
// flight during this tile's math. Per-row side data (row_first, and the backward's lse) come
// the same way (4 B per lane), so the loop carries no register loads. The math is that of the
// register kernels, operand for operand (bitwise-equal results).
// LDS tile: 16 rows x 128 B; 16-B chunk G of row r sits at slot G ^ ((r >> 1) & 7), so the
// 16 lanes reading one chunk of rows 0..15 hit 16 distinct slots of the 256-B bank row.
__device__ __forceinline__ int tsw(int r) { return (r >> 1) & 7; }

__device__ __forceinline__ void glds_b(const void* src, void* lds, int bytes) {
  if (bytes == 16)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
  else
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
}

// one head slice (64 x 16-bit) of tile rows t0 .. t0+15 (clamped to n-1) into a 2-KB LDS tile
template <typename T>
__device__ __forceinline__ void stage_slice(const T* col, int ld, int row0, int n, char* dst, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rr = 8 * i + (lane >> 3), c = (lane & 7) ^ tsw(rr);
    glds_b(col + (size_t)(row0 + min(rr, n - 1)) * ld + 8 * c, dst + i * 1024, 16);
  }
}
// 16-B operand fragment: row r, 16-B chunk G
__device__ __forceinline__ s16x8 lds_frag(const char* tile, int r, int G) {
  return *reinterpret_cast<const s16x8*>(tile + r * 128 + ((G ^ tsw(r)) << 4));
}
// Transposed operand reads (cf. tr_read) of the four 16-column blocks of a tile, and their
// completion, in one asm statement. Issued through the ds_read_tr intrinsic, each read gets a
// vmcnt(0) in front of it from the compiler (it cannot tell the read from the in-flight
// global_load_lds of the next ring slot), which would drain the prefetch every tile.
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ void tr_read4_at(const uint32_t (&a)[4], s16x4 (&r)[4]) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %4\n\t"
      "ds_read_b64_tr_b16 %1, %5\n\t"
      "ds_read_b64_tr_b16 %2, %6\n\t"
      "ds_read_b64_tr_b16 %3, %7\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3])
      : "memory");
}
// swizzled 2-KB ring tile, rows rbase..rbase+3 per lane group (rbase = 4 g4)
__device__ __forceinline__ void tr_read4_sw(const char* tile, int rbase, int lane, s16x4 (&r)[4]) {
  const int li = lane & 15, row = rbase + (li >> 2);
  uint32_t a[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int col = 16 * t + 4 * (li & 3);
    a[t] = lds_off(tile + row * 128 + (((col >> 3) ^ tsw(row)) << 4) + (col & 7) * 2);
  }
  tr_read4_at(a, r);
}
// padded TRS tile (the prefix K / V staged once per wave)
__device__ __forceinline__ void tr_read4_pad(const short* tile, int rbase, int lane, s16x4 (&r)[4]) {
  const int li = lane & 15;
  uint32_t a[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) a[t] = lds_off(tile + (rbase + (li >> 2)) * TRS + 16 * t + 4 * (li & 3));
  tr_read4_at(a, r);
}

template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <typename T, int NS, int WPB>
__global__ __launch_bounds__(WPB * 64) void attn_prefix_fwd_lds(int G, int P, int R, int ntiles,
                                                           const int* __restrict__ tiles,
                                                           const int* __restrict__ row_first, int H,
                                                           int nchunk, int uc, const T* __restrict__ qkv,
                                                           int ldq, T* __restrict__ out, int ldo,
                                                           float* __restrict__ lse, int cls0) {
  constexpr int SLOT = 3 * 2048 + 256;  // q | k | v tiles, row_first of the 16 rows (+ lane copies)
  constexpr int PER = 7;                // global_load_lds per tile
  __shared__ CLIPK_LDS_ALIGN char sm[WPB][NS * SLOT + 16 * TRS * 2];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int wid = blockIdx.x * WPB + w;
  if (wid >= G * nchunk * H) return;  // wave-uniform; no block barriers below
  const int h = wid % H, k = (wid / H) % nchunk, g = wid / (H * nchunk);
  const int W = H * 64;
  char* ring = sm[w];
  short* sVp = reinterpret_cast<short*>(ring + NS * SLOT);
  const int gR = g * R;
  const T* qh = qkv + h * 64;
  const int u_begin = k * uc, u_end = min((k + 1) * uc, ntiles + 1);
  const int tab = load_tile_table(tiles, ntiles, u_begin, lane);
  auto issue = [&](int u, int slot) {
    int t0, n, pre;
    tile_info(tab, P, u, u_begin, t0, n, pre);
    char* b = ring + slot * SLOT;
#pragma unroll
    for (int j = 0; j < 3; ++j) stage_slice<T>(qh + j * W, ldq, (cls0 && u > 0 ? 0 : gR) + t0, n, b + j * 2048, lane);
    glds_b(row_first + t0 + min(r16, n - 1), b + 3 * 2048, 4);
  };
  const bool pok = r16 < P;
  const T* pp = qh + (gR + (pok ? r16 : 0)) * ldq;
  s16x8 kp[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int c = 8 * g4 + 32 * kk;
    kp[kk] = ld_row16(pp + W + c, pok);
    *reinterpret_cast<s16x8*>(sVp + r16 * TRS + c) = ld_row16(pp + 2 * W + c, pok);
  }
  const int nu = u_end - u_begin;
#pragma unroll
  for (int d = 0; d < NS - 1; ++d)
    if (d < nu) issue(u_begin + d, d);
  for (int i = 0; i < nu; ++i) {
    const int u = u_begin + i;
    // ring: tile i+NS-1 goes into the slot tile i-1 was read from (its reads retired)
    lds_fence();
    if (i + NS - 1 < nu) issue(u + NS - 1, (i + NS - 1) % NS);
    const int ahead = min(NS - 1, nu - 1 - i);  // tiles issued after tile i
    if (ahead >= 2) vm_wait<2 * PER>();
    else if (ahead == 1) vm_wait<PER>();
    else vm_wait<0>();
    const char* b = ring + (i % NS) * SLOT;
    int t0, n, pre;
    tile_info(tab, P, u, u_begin, t0, n, pre);
    const int first = u == 0 ? 0 : reinterpret_cast<const int*>(b + 3 * 2048)[r16] - t0;
    const bool qok = r16 < n;
    s16x8 q[2], ko[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      q[kk] = lds_frag(b, r16, g4 + 4 * kk);
      ko[kk] = lds_frag(b + 2048, r16, g4 + 4 * kk);
    }
    f32x4 sp = {0.f, 0.f, 0.f, 0.f}, so = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      sp = mfma32_t<T>(kp[kk], q[kk], sp);
      so = mfma32_t<T>(ko[kk], q[kk], so);
    }
    float vp[4], vq[4], mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = 4 * g4 + r;
      vp[r] = key < pre ? sp[r] * kScale : -INFINITY;
      vq[r] = (key <= r16 && key >= first) ? so[r] * kScale : -INFINITY;
      mx = fmaxf(mx, fmaxf(vp[r], vq[r]));
    }
    mx = xmax4(mx);
    float ep[4], eo[4], ps = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ep[r] = __expf(vp[r] - mx);
      eo[r] = __expf(vq[r] - mx);
      ps += ep[r] + eo[r];
    }
    ps = xsum4(ps);
    const s16x4 bp = pack4<T>(ep[0], ep[1], ep[2], ep[3]);
    const s16x4 bo = pack4<T>(eo[0], eo[1], eo[2], eo[3]);
    const float inv = 1.0f / ps;
    s16x4 tp[4], to[4];
    tr_read4_pad(sVp, 4 * g4, lane, tp);
    tr_read4_sw(b + 2 * 2048, 4 * g4, lane, to);
    f32x4 o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      o[t] = mfma16_t<T>(tp[t], bp, (f32x4){0.f, 0.f, 0.f, 0.f});
      o[t] = mfma16_t<T>(to[t], bo, o[t]);
    }
    store_tile64<T>(out + (gR + t0 + r16) * ldo + h * 64, o, inv, qok);
    if (lse && g4 == 0 && qok) lse[(gR + t0 + r16) * H + h] = mx + __logf(ps);
  }
}

template <typename T, int NS, int WPB>
__global__ __launch_bounds__(WPB * 64) void attn_prefix_bwd_lds(int G, int P, int R, int ntiles,
                                                           const int* __restrict__ tiles,
                                                           const int* __restrict__ row_first, int H,
                                                           int nchunk, int uc, const T* __restrict__ qkv,
                                                           int ldq, const T* __restrict__ dout, int lddo,
                                                           const float* __restrict__ lse,
                                                           T* __restrict__ dqkv, int lddq,
                                                           float* __restrict__ part, int cls0) {
  static_assert(sizeof(T) == 2, "MFMA attention backward: 16-bit operands");
  constexpr int SLOT = 4 * 2048 + 2 * 256;  // q | k | v | dO tiles, row_first, lse
  constexpr int PER = 10;
  __shared__ CLIPK_LDS_ALIGN char sm[WPB][NS * SLOT + 16 * TRS * 2];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int wid = blockIdx.x * WPB + w;
  if (wid >= G * nchunk * H) return;  // wave-uniform
  const int h = wid % H, k = (wid / H) % nchunk, g = wid / (H * nchunk);
  const int W = H * 64;
  char* ring = sm[w];
  short* tKp = reinterpret_cast<short*>(ring + NS * SLOT);
  const int gR = g * R;
  const T* qh = qkv + h * 64;
  const int u_begin = k * uc, u_end = min((k + 1) * uc, ntiles + 1);
  const int tab = load_tile_table(tiles, ntiles, u_begin, lane);
  auto issue = [&](int u, int slot) {
    int t0, n, pre;
    tile_info(tab, P, u, u_begin, t0, n, pre);
    char* b = ring + slot * SLOT;
#pragma unroll
    for (int j = 0; j < 3; ++j) stage_slice<T>(qh + j * W, ldq, (cls0 && u > 0 ? 0 : gR) + t0, n, b + j * 2048, lane);
    stage_slice<T>(dout + h * 64, lddo, gR + t0, n, b + 3 * 2048, lane);
    const int rr = t0 + min(r16, n - 1);
    glds_b(row_first + rr, b + 4 * 2048, 4);
    glds_b(lse + (size_t)(gR + rr) * H + h, b + 4 * 2048 + 256, 4);
  };
  const bool pok = r16 < P;
  const T* pp = qh + (gR + (pok ? r16 : 0)) * ldq;
  s16x8 kp[2], vp[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int c = 8 * g4 + 32 * kk;
    kp[kk] = ld_row16(pp + W + c, pok);
    vp[kk] = ld_row16(pp + 2 * W + c, pok);
    *reinterpret_cast<s16x8*>(tKp + r16 * TRS + c) = kp[kk];
  }
  f32x4 dkp[4], dvp[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    dkp[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    dvp[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  const int nu = u_end - u_begin;
#pragma unroll
  for (int d = 0; d < NS - 1; ++d)
    if (d < nu) issue(u_begin + d, d);
  for (int i = 0; i < nu; ++i) {
    const int u = u_begin + i;
    lds_fence();
    if (i + NS - 1 < nu) issue(u + NS - 1, (i + NS - 1) % NS);
    const int ahead = min(NS - 1, nu - 1 - i);
    if (ahead >= 2) vm_wait<2 * PER>();
    else if (ahead == 1) vm_wait<PER>();
    else vm_wait<0>();
    const char* b = ring + (i % NS) * SLOT;
    const char* tQ = b;
    const char* tKo = b + 2048;
    const char* tD = b + 3 * 2048;
    const int* sF = reinterpret_cast<const int*>(b + 4 * 2048);
    const float* sL = reinterpret_cast<const float*>(b + 4 * 2048 + 256);
    int t0, n, pre;
    tile_info(tab, P, u, u_begin, t0, n, pre);
    const bool own_is_prefix = u == 0;
    const bool qok = r16 < n;
    s16x8 q[2], ko[2], vo[2], d[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      q[kk] = lds_frag(tQ, r16, g4 + 4 * kk);
      ko[kk] = lds_frag(tKo, r16, g4 + 4 * kk);
      vo[kk] = lds_frag(b + 2 * 2048, r16, g4 + 4 * kk);
      d[kk] = lds_frag(tD, r16, g4 + 4 * kk);
    }
    const float l2 = sL[r16];
    const int first2 = own_is_prefix ? 0 : sF[r16] - t0;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    f32x4 s1p = z, s2p = z, p1p = z, p2p = z, s1o = z, s2o = z, p1o = z, p2o = z;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      s1p = mfma32_t<T>(q[kk], kp[kk], s1p);
      s2p = mfma32_t<T>(kp[kk], q[kk], s2p);
      p1p = mfma32_t<T>(d[kk], vp[kk], p1p);
      p2p = mfma32_t<T>(vp[kk], d[kk], p2p);
      s1o = mfma32_t<T>(q[kk], ko[kk], s1o);
      s2o = mfma32_t<T>(ko[kk], q[kk], s2o);
      p1o = mfma32_t<T>(d[kk], vo[kk], p1o);
      p2o = mfma32_t<T>(vo[kk], d[kk], p2o);
    }
    float P2p[4], P2o[4], Dsum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 4 * g4 + r;
      P2p[r] = (qok && j < pre) ? __expf(s2p[r] * kScale - l2) : 0.f;
      P2o[r] = (qok && j <= r16 && j >= first2) ? __expf(s2o[r] * kScale - l2) : 0.f;
      Dsum += P2p[r] * p2p[r] + P2o[r] * p2o[r];
    }
    Dsum = xsum4(Dsum);
    float dS2p[4], dS2o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dS2p[r] = P2p[r] * (p2p[r] - Dsum);
      dS2o[r] = P2o[r] * (p2o[r] - Dsum);
    }
    float P1p[4], P1o[4], dS1p[4], dS1o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i4 = 4 * g4 + r;
      const bool iok = i4 < n;
      const float Di = __shfl(Dsum, i4, 64);
      const float l1 = sL[i4];
      const int first1 = own_is_prefix ? 0 : sF[i4] - t0;
      P1p[r] = (iok && r16 < pre) ? __expf(s1p[r] * kScale - l1) : 0.f;
      P1o[r] = (iok && r16 <= i4 && r16 >= first1) ? __expf(s1o[r] * kScale - l1) : 0.f;
      dS1p[r] = P1p[r] * (p1p[r] - Di);
      dS1o[r] = P1o[r] * (p1o[r] - Di);
    }
    const s16x4 bPp = pack4<T>(P1p[0], P1p[1], P1p[2], P1p[3]);
    const s16x4 bSp = pack4<T>(dS1p[0], dS1p[1], dS1p[2], dS1p[3]);
    const s16x4 bPo = pack4<T>(P1o[0], P1o[1], P1o[2], P1o[3]);
    const s16x4 bSo = pack4<T>(dS1o[0], dS1o[1], dS1o[2], dS1o[3]);
    const s16x4 bTp = pack4<T>(dS2p[0], dS2p[1], dS2p[2], dS2p[3]);
    const s16x4 bTo = pack4<T>(dS2o[0], dS2o[1], dS2o[2], dS2o[3]);
    T* orow = dqkv + (gR + t0 + r16) * lddq + h * 64;
    f32x4 acc[4];
    s16x4 ta[4], tb[4];
    tr_read4_pad(tKp, 4 * g4, lane, ta);
    tr_read4_sw(tKo, 4 * g4, lane, tb);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[t] = mfma16_t<T>(ta[t], bTp, z);
      acc[t] = mfma16_t<T>(tb[t], bTo, acc[t]);
    }
    store_tile64<T>(orow, acc, kScale, qok);  // dQ
    tr_read4_sw(tQ, 4 * g4, lane, ta);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const s16x4 aQ = ta[t];
      dkp[t] = mfma16_t<T>(aQ, bSp, dkp[t]);
      acc[t] = mfma16_t<T>(aQ, bSo, z);
      if (own_is_prefix) dkp[t] += acc[t];
    }
    if (!own_is_prefix) store_tile64<T>(orow + W, acc, kScale, qok);  // dK
    tr_read4_sw(tD, 4 * g4, lane, tb);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const s16x4 aD = tb[t];
      dvp[t] = mfma16_t<T>(aD, bPp, dvp[t]);
      acc[t] = mfma16_t<T>(aD, bPo, z);
      if (own_is_prefix) dvp[t] += acc[t];
    }
    if (!own_is_prefix) store_tile64<T>(orow + 2 * W, acc, 1.0f, qok);  // dV
  }
  float* pb = part + ((size_t)g * nchunk + k) * 16 * (2 * W);
  if (r16 < P) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float* dst = pb + (size_t)r16 * 2 * W + h * 64 + 16 * t + 4 * g4;
      *reinterpret_cast<f32x4*>(dst) = dkp[t] * kScale;
      *reinterpret_cast<f32x4*>(dst + W) = dvp[t];
    }
  }
}

// ------------------------------------------------------------------ fp32 kernels (PREC fp32 / fp32s)
// One wave per (group, chunk of f32_uc units, head); blocks of WPB waves (f32_wpb) share one
// (group, head), so the prefix K/V rows are staged into LDS once per block. Lane = 4 r + s: row
// r of the unit (query in the forward and for dQ, key for dK / dV) and 16-column slice s of
// the head; a dot product is 16 FMAs on the lane's slice plus a quad sum (2 DPP adds). K/V
// (and, for the backward's key phases, Q / dO) rows are read from LDS, where the 16 lanes of
// one slice read the same 64 B (a broadcast). All arithmetic fp32, the reference's
// nn.MultiheadAttention math (model.py:183), exact softmax (online max / rescale, fwd).
// waves per block (template WPB; knob CLIPK_F32ATTN_WPB: 2 (default), 4 or 8). fp32s headline
// (profiles/r04h/): backward 2.86 -> 2.76 ms/step at 2 vs 4, forward equal, 8 no better
static int f32_wpb() { static int c = chunk_env("CLIPK_F32ATTN_WPB", 2); return c == 4 || c == 8 ? c : 2; }

// a wave's own LDS writes visible to its other lanes (program order on the LDS; no reordering
// by the compiler across this point)
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// unit u of group-relative tiles: first row t0, rows n (<= 16), prefix keys pre, and for row rr
// the first row of its class (causal block-diagonal mask inside the tile)
__device__ __forceinline__ void f32_unit(const int* __restrict__ tiles, const int* __restrict__ row_first, int P,
                                         int u, int r, int& t0, int& n, int& pre, int& rr, int& first) {
  if (u == 0) {
    t0 = 0; n = P; pre = 0;
  } else {
    t0 = tiles[2 * (u - 1)];
    n = min(tiles[2 * (u - 1) + 1], 16);
    pre = P;
  }
  rr = min(r, n - 1);
  first = u == 0 ? 0 : row_first[t0 + rr] - t0;
}

// block (g, h, chunk block kb): waves take chunks kb * WPB + w; stages the prefix K / V rows
// of (g, h) (P <= 16 rows x 64 fp32) into sKp / sVp. These sit in DYNAMIC LDS sized to P rows
// (2 x P x 256 B, f32_prefix_lds): at the CoCoOp P of 5 a block takes 2.5 KiB for them instead of
// 8, which lets 5 backward blocks (10 waves) and 8 forward blocks (16 waves) share a CU instead
// of 4 and 6 (LDS was the occupancy limit: 34 / 24 KiB per 2-wave block)
template <int WPB>
__device__ __forceinline__ void f32_block(int H, int nchunk, int& g, int& h, int& k, int& w) {
  const int nkb = (nchunk + WPB - 1) / WPB;
  const int b = blockIdx.x;
  h = b % H;
  const int kb = (b / H) % nkb;
  g = b / (H * nkb);
  w = threadIdx.x >> 6;
  k = kb * WPB + w;
}
template <int WPB>
__device__ __forceinline__ void f32_stage_prefix(const float* __restrict__ qkv, size_t row0, int P, int ldq, int col,
                                                 int W, float* sKp, float* sVp) {
  for (int i = threadIdx.x; i < P * 16; i += WPB * 64) {  // P rows x 16 float4
    const int j = i >> 4, c = i & 15;
    const float* b = qkv + (row0 + j) * ldq + col + 4 * c;
    reinterpret_cast<f32x4*>(sKp)[i] = *reinterpret_cast<const f32x4*>(b + W);
    reinterpret_cast<f32x4*>(sVp)[i] = *reinterpret_cast<const f32x4*>(b + 2 * W);
  }
}
static size_t f32_prefix_lds(int P) { return (size_t)2 * P * 64 * sizeof(float); }

template <int WPB>
__global__ __launch_bounds__(WPB * 64) void attn_prefix_fwd_f32(
    int G, int P, int R, int ntiles, const int* __restrict__ tiles, const int* __restrict__ row_first, int H,
    int nchunk, int uc, const float* __restrict__ qkv, int ldq, float* __restrict__ out, int ldo,
    float* __restrict__ lse, int cls0) {
  extern __shared__ CLIPK_LDS_ALIGN float sPre[];  // prefix K | V rows, P x 64 each (f32_prefix_lds)
  float* const sKp = sPre;
  float* const sVp = sPre + P * 64;
  __shared__ CLIPK_LDS_ALIGN float sK[WPB][16 * 64], sV[WPB][16 * 64];
  int g, h, k, w;
  f32_block<WPB>(H, nchunk, g, h, k, w);
  const int W = H * 64;
  f32_stage_prefix<WPB>(qkv, (size_t)g * R, P, ldq, h * 64, W, sKp, sVp);
  __syncthreads();
  if (k >= nchunk) return;  // wave-uniform; no block barrier follows
  const int lane = threadIdx.x & 63, r = lane >> 2, s = lane & 3;
  float* sk = sK[w];
  float* sv = sV[w];
  const int u_end = min((k + 1) * uc, ntiles + 1);
  // the next unit's q / k / v rows are loaded into registers while this unit computes (one
  // unit ahead: a wave otherwise waits out a full HBM latency per unit)
  float qn[16], kn[16], vn[16];
  int t0n, nn, pren, rrn, firstn;
  auto fetch = [&](int u) {
    f32_unit(tiles, row_first, P, u, r, t0n, nn, pren, rrn, firstn);
    const float* qp = qkv + ((cls0 && u > 0 ? 0 : (size_t)g * R) + t0n + rrn) * ldq + h * 64 + kSl * s;
    ld16x(qp, qn);
    ld16x(qp + W, kn);
    ld16x(qp + 2 * W, vn);
  };
  if (k * uc < u_end) fetch(k * uc);
  for (int u = k * uc; u < u_end; ++u) {
    const int t0 = t0n, n = nn, pre = pren, rr = rrn, first = firstn;
    const size_t row = (size_t)g * R + t0 + rr;
    float q[16];
#pragma unroll
    for (int d = 0; d < 16; ++d) q[d] = qn[d] * kScale;
    st16x(sk + r * 64 + kSl * s, kn);
    st16x(sv + r * 64 + kSl * s, vn);
    lds_sync();
    if (u + 1 < u_end) fetch(u + 1);
    // exact two-pass softmax over the prefix keys, then the row's own class keys first..rr: the
    // scores stay in registers (key loops unrolled to 16 with wave-uniform bounds), so there is
    // no per-key rescale branch (the online form diverged per row on every new maximum)
    float sp[16], so[16], m = -INFINITY;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j < pre) {
        float kv[16];
        ld16x(sKp + j * 64 + kSl * s, kv);
        sp[j] = quad_sum(dot16(q, kv));
        m = fmaxf(m, sp[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j < n) {
        float kv[16];
        ld16x(sk + j * 64 + kSl * s, kv);
        const float sc = quad_sum(dot16(q, kv));
        so[j] = (j <= rr && j >= first) ? sc : -INFINITY;
        m = fmaxf(m, so[j]);
      }
    }
    float l = 0.f, o[16];
#pragma unroll
    for (int d = 0; d < 16; ++d) o[d] = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j < pre) {
        float vv[16];
        ld16x(sVp + j * 64 + kSl * s, vv);
        const float p = __expf(sp[j] - m);
        l += p;
#pragma unroll
        for (int d = 0; d < 16; ++d) o[d] = fmaf(p, vv[d], o[d]);
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j < n) {
        float vv[16];
        ld16x(sv + j * 64 + kSl * s, vv);
        const float p = __expf(so[j] - m);  // 0 for the masked keys
        l += p;
#pragma unroll
        for (int d = 0; d < 16; ++d) o[d] = fmaf(p, vv[d], o[d]);
      }
    }
    if (r < n) {
      const float inv = 1.0f / l;
#pragma unroll
      for (int d = 0; d < 16; ++d) o[d] *= inv;
      st16x(out + row * ldo + h * 64 + kSl * s, o);
      if (lse && s == 0) lse[row * H + h] = m + __logf(l);
    }
    lds_sync();  // this unit's sK / sV reads done before the next unit's writes (program order)
  }
}

// Backward per unit: phase 1 (lane = query): P, dS over the prefix + own keys, dQ; P / dS kept in
// LDS ([16 queries][16 prefix | 16 own keys], zero where masked). Phase 2 (lane = own key):
// dK, dV over the unit's queries (the prefix unit's own keys ARE the prefix rows: accumulated).
// Phase 3 (lane = prefix key): the prefix rows' dK, dV partial of this unit, accumulated over
// the chunk in registers and written once per chunk (prefix_kv_reduce sums the chunks).
// OS (grad dtype CLIPK_F32S): dQ / dK / dV stored in the pre-split form of the qkv input-grad
// GEMM's A (st16x_split; the prefix rows' dK / dV by prefix_kv_reduce_split), the same bytes
template <int WPB, bool OS = false>
__global__ __launch_bounds__(WPB * 64, 2) void attn_prefix_bwd_f32(  // >= 2 waves per SIMD (<= 256 VGPRs)
    int G, int P, int R, int ntiles, const int* __restrict__ tiles, const int* __restrict__ row_first, int H,
    int nchunk, int uc, const float* __restrict__ qkv, int ldq, const float* __restrict__ o_fwd, int ldof,
    const float* __restrict__ dout, int lddo, const float* __restrict__ lse, float* __restrict__ dqkv, int lddq,
    float* __restrict__ part, int cls0) {
  extern __shared__ CLIPK_LDS_ALIGN float sPre[];  // prefix K | V rows, P x 64 each (f32_prefix_lds)
  float* const sKp = sPre;
  float* const sVp = sPre + P * 64;
  // padded rows (bank-conflict-free stores): K|V then Q|dO rows at stride RS floats; P / dS at
  // stride PS (a column of 16 query rows written by one lane per row hit 2 banks at stride 32)
  constexpr int RS = 68, PS = 33;
  __shared__ CLIPK_LDS_ALIGN float sA[WPB][16 * RS], sB[WPB][16 * RS];
  __shared__ CLIPK_LDS_ALIGN float sP[WPB][16 * PS], sS[WPB][16 * PS];
  int g, h, k, w;
  f32_block<WPB>(H, nchunk, g, h, k, w);
  const int W = H * 64;
  f32_stage_prefix<WPB>(qkv, (size_t)g * R, P, ldq, h * 64, W, sKp, sVp);
  __syncthreads();
  if (k >= nchunk) return;
  const int lane = threadIdx.x & 63, r = lane >> 2, s = lane & 3;
  float* sa = sA[w];
  float* sb = sB[w];
  float* sp = sP[w];
  float* ss = sS[w];
  float akp[16], avp[16];  // prefix row r's dK / dV slice, summed over the chunk
#pragma unroll
  for (int d = 0; d < 16; ++d) { akp[d] = 0.f; avp[d] = 0.f; }
  const int u_end = min((k + 1) * uc, ntiles + 1);
  // the next unit's rows (q, dO, o, k, v, lse) are loaded into registers while this unit
  // computes (one unit ahead, as the forward)
  float qn[16], dOn[16], on[16], kn[16], vn[16], lin = 0.f;
  int t0n, nn, pren, rrn, firstn;
  auto fetch = [&](int u) {
    f32_unit(tiles, row_first, P, u, r, t0n, nn, pren, rrn, firstn);
    const size_t rw = (size_t)g * R + t0n + rrn;
    const float* qp = qkv + ((cls0 && u > 0 ? 0 : (size_t)g * R) + t0n + rrn) * ldq + h * 64 + kSl * s;
    ld16x(qp, qn);
    ld16x(dout + rw * lddo + h * 64 + kSl * s, dOn);
    ld16x(o_fwd + rw * ldof + h * 64 + kSl * s, on);
    ld16x(qp + W, kn);
    ld16x(qp + 2 * W, vn);
    lin = lse[rw * H + h];
  };
  if (k * uc < u_end) fetch(k * uc);
  for (int u = k * uc; u < u_end; ++u) {
    const int t0 = t0n, n = nn, pre = pren, rr = rrn, first = firstn;
    const bool qok = r < n;
    const size_t row = (size_t)g * R + t0 + rr;
    float q[16], dO[16];
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      q[d] = qn[d] * kScale;
      dO[d] = dOn[d];
    }
    const float Di = quad_sum(dot16(dO, on));
    const float li = lin;
    st16x(sa + r * RS + kSl * s, kn);
    st16x(sb + r * RS + kSl * s, vn);
    lds_sync();
    if (u + 1 < u_end) fetch(u + 1);
    // phase 1: lane = query row rr
    float dq[16];
#pragma unroll
    for (int d = 0; d < 16; ++d) dq[d] = 0.f;
    auto key = [&](const float* kr, const float* vr, bool ok, int col) {
      float kv[16], vv[16];
      ld16x(kr + kSl * s, kv);
      ld16x(vr + kSl * s, vv);
      const float sc = quad_sum(dot16(q, kv));
      const float dp = quad_sum(dot16(dO, vv));
      const float p = ok ? __expf(sc - li) : 0.f;
      const float ds = p * (dp - Di);
#pragma unroll
      for (int d = 0; d < 16; ++d) dq[d] = fmaf(ds, kv[d], dq[d]);
      if (s == 0) {
        sp[r * PS + col] = p;
        ss[r * PS + col] = ds;
      }
    };
    for (int j = 0; j < pre; ++j) key(sKp + j * 64, sVp + j * 64, qok, j);
    for (int j = 0; j < n; ++j) key(sa + j * RS, sb + j * RS, qok && j <= rr && j >= first, 16 + j);
    if (qok) {
#pragma unroll
      for (int d = 0; d < 16; ++d) dq[d] *= kScale;
      if constexpr (OS) st16x_split(dqkv + row * lddq + h * 64 + kSl * s, dq, s);
      else st16x(dqkv + row * lddq + h * 64 + kSl * s, dq);
    }
    // sA / sB: the unit's scaled q and dO rows for the key phases (after every lane's phase-1
    // reads of K / V: program order)
    st16x(sa + r * RS + kSl * s, q);
    st16x(sb + r * RS + kSl * s, dO);
    lds_sync();
    // phases 2 / 3: lane = key; sum over the unit's queries i of dS[i][key] q_i, P[i][key] dO_i
    auto keysum = [&](int col, float* dk, float* dv) {
      for (int i = 0; i < n; ++i) {
        const float pv = sp[i * PS + col], dsv = ss[i * PS + col];
        float a[16], b[16];
        ld16x(sa + i * RS + kSl * s, a);
        ld16x(sb + i * RS + kSl * s, b);
#pragma unroll
        for (int d = 0; d < 16; ++d) {
          dk[d] = fmaf(dsv, a[d], dk[d]);
          dv[d] = fmaf(pv, b[d], dv[d]);
        }
      }
    };
    if (u == 0) {  // the prefix unit: its own keys are the prefix rows
      keysum(16 + r, akp, avp);
    } else {
      float dk[16], dv[16];
#pragma unroll
      for (int d = 0; d < 16; ++d) { dk[d] = 0.f; dv[d] = 0.f; }
      // own key 16 + r and prefix key r in one pass over the unit's queries: each q / dO row is
      // read from LDS once for both (the same per-accumulator FMA order as two keysum passes)
      for (int i = 0; i < n; ++i) {
        const float pv = sp[i * PS + 16 + r], dsv = ss[i * PS + 16 + r];
        const float pp = sp[i * PS + r], dsp = ss[i * PS + r];
        float a[16], b[16];
        ld16x(sa + i * RS + kSl * s, a);
        ld16x(sb + i * RS + kSl * s, b);
#pragma unroll
        for (int d = 0; d < 16; ++d) {
          dk[d] = fmaf(dsv, a[d], dk[d]);
          dv[d] = fmaf(pv, b[d], dv[d]);
          akp[d] = fmaf(dsp, a[d], akp[d]);
          avp[d] = fmaf(pp, b[d], avp[d]);
        }
      }
      if (qok) {
        if constexpr (OS) {
          st16x_split(dqkv + row * lddq + W + h * 64 + kSl * s, dk, s);
          st16x_split(dqkv + row * lddq + 2 * W + h * 64 + kSl * s, dv, s);
        } else {
          st16x(dqkv + row * lddq + W + h * 64 + kSl * s, dk);
          st16x(dqkv + row * lddq + 2 * W + h * 64 + kSl * s, dv);
        }
      }
    }
    lds_sync();
  }
  if (r < P) {
    // (dK = sum dS q with q already scaled: no further factor)
    float* pb = part + (((size_t)g * nchunk + k) * 16 + r) * (2 * W) + h * 64 + kSl * s;
    st16x(pb, akp);
    st16x(pb + W, avp);
  }
}

// prefix rows' dK | dV = sum over chunks of the partials (fixed order)
template <typename TG>
__global__ __launch_bounds__(256) void prefix_kv_reduce(int P, int R, int W, int nchunk,
                                                        const float* __restrict__ part,
                                                        TG* __restrict__ dqkv, int lddq) {
  const int g = blockIdx.x / P, p = blockIdx.x % P;
  const int col = blockIdx.y * 256 + threadIdx.x;
  if (col >= 2 * W) return;
  const float* src = part + ((size_t)g * nchunk * 16 + p) * 2 * W + col;
  const size_t cs = (size_t)16 * 2 * W;  // chunk stride
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;  // 4 independent chains, fixed order
  int k = 0;
  // 16 chunks' loads in flight per round trip (the sums keep the 4-chain order)
  for (; k + 16 <= nchunk; k += 16) {
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = src[(k + i) * cs];
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
      a0 += v[i];
      a1 += v[i + 1];
      a2 += v[i + 2];
      a3 += v[i + 3];
    }
  }
  for (; k + 4 <= nchunk; k += 4) {
    a0 += src[k * cs];
    a1 += src[(k + 1) * cs];
    a2 += src[(k + 2) * cs];
    a3 += src[(k + 3) * cs];
  }
  for (; k < nchunk; ++k) a0 += src[k * cs];
  const float acc = (a0 + a1) + (a2 + a3);
  dqkv[((size_t)g * R + p) * lddq + W + col] = (TG)acc;
}

// prefix_kv_reduce for the pre-split dQ|dK|dV (grad dtype CLIPK_F32S): column col's fp16 hi / lo
// parts at byte 2 (col % 8) of its 8-column group's hi / lo halves (the same sums, fixed order)
__global__ __launch_bounds__(256) void prefix_kv_reduce_split(int P, int R, int W, int nchunk,
                                                              const float* __restrict__ part,
                                                              float* __restrict__ dqkv, int lddq) {
  const int g = blockIdx.x / P, p = blockIdx.x % P;
  const int col = blockIdx.y * 256 + threadIdx.x;
  if (col >= 2 * W) return;
  const float* src = part + ((size_t)g * nchunk * 16 + p) * 2 * W + col;
  const size_t cs = (size_t)16 * 2 * W;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;  // prefix_kv_reduce's chains and order
  int k = 0;
  for (; k + 16 <= nchunk; k += 16) {
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = src[(k + i) * cs];
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
      a0 += v[i];
      a1 += v[i + 1];
      a2 += v[i + 2];
      a3 += v[i + 3];
    }
  }
  for (; k + 4 <= nchunk; k += 4) {
    a0 += src[k * cs];
    a1 += src[(k + 1) * cs];
    a2 += src[(k + 2) * cs];
    a3 += src[(k + 3) * cs];
  }
  for (; k < nchunk; ++k) a0 += src[k * cs];
  _Float16 hi, lo;
  split_parts((a0 + a1) + (a2 + a3), hi, lo);
  const int c = W + col;  // column within the q|k|v row
  _Float16* grp = reinterpret_cast<_Float16*>(dqkv + ((size_t)g * R + p) * lddq + (c & ~7));
  grp[c & 7] = hi;
  grp[8 + (c & 7)] = lo;
}

template <typename T>
static int prefix_fwd(int G, int P, int R, int ntiles, const int* tiles, const int* row_first, int H,
                      const void* qkv, int ldq, void* out, int ldo, float* lse, hipStream_t st, int cls0) {
  if constexpr (sizeof(T) == 2) {
    const int uc = fwd_chunk();
    const int nchunk = n_chunks(ntiles, uc);
    const long waves = (long)G * nchunk * H;
    if (const int ns = lds_slots()) {
      const int wpb = lds_wpb();
      auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3((waves + wpb - 1) / wpb), dim3(64 * wpb), 0, st, G, P, R, ntiles, tiles,
                           row_first, H, nchunk, uc, (const T*)qkv, ldq, (T*)out, ldo, lse, cls0);
      };
#define CLIPK_LDS_GO(K, T_, ...)                                                               \
  if (ns == 2) { if (wpb == 1) go(K<T_, 2, 1 __VA_ARGS__>); else if (wpb == 2) go(K<T_, 2, 2 __VA_ARGS__>); \
                 else go(K<T_, 2, 4 __VA_ARGS__>); }                                                 \
  else { if (wpb == 1) go(K<T_, 3, 1 __VA_ARGS__>); else if (wpb == 2) go(K<T_, 3, 2 __VA_ARGS__>);     \
         else go(K<T_, 3, 4 __VA_ARGS__>); }
      CLIPK_LDS_GO(attn_prefix_fwd_lds, T)
      CLIPK_CHECK_LAUNCH();
      return CLIPK_OK;
    }
    const int b = fwd_batch();
    const int wpb = prefix_wpb();
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((waves + wpb - 1) / wpb), dim3(64 * wpb), 0, st, G, P, R, ntiles, tiles,
                         row_first, H, nchunk, uc, (const T*)qkv, ldq, (T*)out, ldo, lse, cls0);
    };
    if (wpb == 8) {
      if (b == 1) go(attn_prefix_fwd_mfma<T, 1, 8>);
      else if (b == 2) go(attn_prefix_fwd_mfma<T, 2, 8>);
      else go(attn_prefix_fwd_mfma<T, 4, 8>);
    } else {
      if (b == 1) go(attn_prefix_fwd_mfma<T, 1>);
      else if (b == 2) go(attn_prefix_fwd_mfma<T, 2>);
      else go(attn_prefix_fwd_mfma<T, 4>);
    }
  } else {
    const int uc = f32_uc(G, ntiles, H, kF32FwdWpc);
    const int nchunk = n_chunks(ntiles, uc);
    auto go = [&](auto kern, int wpb) {
      const long blocks = (long)G * ((nchunk + wpb - 1) / wpb) * H;
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * wpb), f32_prefix_lds(P), st, G, P, R, ntiles, tiles, row_first,
                         H, nchunk, uc, (const float*)qkv, ldq, (float*)out, ldo, lse, cls0);
    };
    const int wpb = f32_wpb();
    if (wpb == 2) go(attn_prefix_fwd_f32<2>, 2);
    else if (wpb == 8) go(attn_prefix_fwd_f32<8>, 8);
    else go(attn_prefix_fwd_f32<4>, 4);
  }
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

template <typename T, typename TG, bool OS = false>
static int prefix_bwd(int G, int P, int R, int ntiles, const int* tiles, const int* row_first, int H,
                      const void* qkv, int ldq, const void* ofwd, int ldof, const void* dout, int lddo,
                      const float* lse, void* dqkv, int lddq, float* part, hipStream_t st, int cls0) {
  static_assert(!OS || (sizeof(T) == 4 && sizeof(TG) == 4), "pre-split dQ|dK|dV: the fp32 backward");
  constexpr bool mfma = sizeof(TG) == 2 && sizeof(T) == 2;
  const int uc = mfma ? bwd_uc(G, ntiles, H) : f32_uc(G, ntiles, H, kF32BwdWpc);
  const int nchunk = n_chunks(ntiles, uc);
  const long waves = (long)G * nchunk * H;
  if constexpr (mfma && __is_same(T, TG)) {
    if (const int ns = lds_slots()) {
      const int wpb = lds_wpb();
      auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3((waves + wpb - 1) / wpb), dim3(64 * wpb), 0, st, G, P, R, ntiles, tiles,
                           row_first, H, nchunk, uc, (const T*)qkv, ldq, (const T*)dout, lddo, lse, (T*)dqkv,
                           lddq, part, cls0);
      };
      CLIPK_LDS_GO(attn_prefix_bwd_lds, T)
      CLIPK_CHECK_LAUNCH();
      const int W = H * 64;
      hipLaunchKernelGGL((prefix_kv_reduce<TG>), dim3(G * P, (2 * W + 255) / 256), dim3(256), 0, st, P, R, W,
                         nchunk, part, (TG*)dqkv, lddq);
      CLIPK_CHECK_LAUNCH();
      return CLIPK_OK;
    }
  }
  if constexpr (mfma) {
    const int wpb = prefix_wpb();
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((waves + wpb - 1) / wpb), dim3(64 * wpb), 0, st, G, P, R, ntiles, tiles,
                         row_first, H, nchunk, uc, (const T*)qkv, ldq, (const TG*)dout, lddo, lse, (TG*)dqkv,
                         lddq, part, cls0);
    };
    if (wpb == 8) {
      if (bwd_batch() == 1) go(attn_prefix_bwd_mfma<T, TG, 1, 8>);
      else go(attn_prefix_bwd_mfma<T, TG, 2, 8>);
    } else {
      if (bwd_batch() == 1) go(attn_prefix_bwd_mfma<T, TG, 1>);
      else go(attn_prefix_bwd_mfma<T, TG, 2>);
    }
  } else {
    static_assert(mfma || (sizeof(T) == 4 && sizeof(TG) == 4), "fp32 backward");
    auto go = [&](auto kern, int wpb) {
      const long blocks = (long)G * ((nchunk + wpb - 1) / wpb) * H;
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * wpb), f32_prefix_lds(P), st, G, P, R, ntiles, tiles, row_first,
                         H, nchunk, uc, (const float*)qkv, ldq, (const float*)ofwd, ldof, (const float*)dout, lddo,
                         lse, (float*)dqkv, lddq, part, cls0);
    };
    const int wpb = f32_wpb();
    if (wpb == 2) go(attn_prefix_bwd_f32<2, OS>, 2);
    else if (wpb == 8) go(attn_prefix_bwd_f32<8, OS>, 8);
    else go(attn_prefix_bwd_f32<4, OS>, 4);
  }
  CLIPK_CHECK_LAUNCH();
  const int W = H * 64;
  if constexpr (OS)
    hipLaunchKernelGGL(prefix_kv_reduce_split, dim3(G * P, (2 * W + 255) / 256), dim3(256), 0, st, P, R, W,
                       nchunk, part, (float*)dqkv, lddq);
  else
    hipLaunchKernelGGL((prefix_kv_reduce<TG>), dim3(G * P, (2 * W + 255) / 256), dim3(256), 0, st, P, R, W,
                       nchunk, part, (TG*)dqkv, lddq);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

}  // namespace clipk

using namespace clipk;

static int prefix_shape_ok(int G, int P, int R, int ntiles, int heads, int ldq) {
  return G > 0 && P >= 1 && P <= 16 && ntiles >= 1 && R > P && heads > 0 &&
         (long)G * R * (long)(ldq > 3 * heads * 64 ? ldq : 3 * heads * 64) < (1L << 31);  // int32 offsets
}

extern "C" size_t clipk_attention_prefix_ws_bytes(int G, int ntiles, int heads) {
  if (G <= 0 || ntiles <= 0 || heads <= 0) return 0;
  const int ub = bwd_uc(G, ntiles, heads), uf = f32_uc(G, ntiles, heads, kF32BwdWpc);
  const int uc = ub < uf ? ub : uf;  // the larger chunk count (16-bit or fp32 backward)
  return (size_t)G * n_chunks(ntiles, uc) * 16 * 2 * heads * 64 * sizeof(float);
}

// flags (the _ex entry points): CLIPK_PREFIX_CLS_GROUP0 -- the class rows' q|k|v are read from
// group 0 for every group (the text encoder's layer 0, whose class rows are the same in every
// group: no per-group copies of them are materialised); prefix rows and every output per group
static int prefix_fwd_call(int dtype, int G, int P, int R, int ntiles, const int* tiles, const int* row_first,
                           int heads, const void* qkv, int ldqkv, void* out, int ldo, float* lse, int flags,
                           void* stream) {
  if (!tiles || !row_first || !qkv || !out) return CLIPK_EINVAL;
  if (flags & ~CLIPK_PREFIX_CLS_GROUP0) return CLIPK_EINVAL;
  if (!prefix_shape_ok(G, P, R, ntiles, heads, ldqkv) || ldqkv < 3 * heads * 64 || ldo < heads * 64 ||
      ldqkv % 8 || ldo % 8)
    return CLIPK_ESHAPE;
  hipStream_t st = (hipStream_t)stream;
  const int c0 = (flags & CLIPK_PREFIX_CLS_GROUP0) ? 1 : 0;
  switch (dtype) {
    case CLIPK_F16: return prefix_fwd<f16>(G, P, R, ntiles, tiles, row_first, heads, qkv, ldqkv, out, ldo, lse, st, c0);
    case CLIPK_BF16: return prefix_fwd<bf16>(G, P, R, ntiles, tiles, row_first, heads, qkv, ldqkv, out, ldo, lse, st, c0);
    case CLIPK_F32: return prefix_fwd<float>(G, P, R, ntiles, tiles, row_first, heads, qkv, ldqkv, out, ldo, lse, st, c0);
    default: return CLIPK_EDTYPE;
  }
}

extern "C" int clipk_attention_prefix_fwd(int dtype, int G, int P, int R, int ntiles, const int* tiles,
                                          const int* row_first, int heads, const void* qkv, int ldqkv,
                                          void* out, int ldo, float* lse, void* stream) {
  return prefix_fwd_call(dtype, G, P, R, ntiles, tiles, row_first, heads, qkv, ldqkv, out, ldo, lse, 0, stream);
}

extern "C" int clipk_attention_prefix_fwd_ex(int dtype, int G, int P, int R, int ntiles, const int* tiles,
                                             const int* row_first, int heads, const void* qkv, int ldqkv,
                                             void* out, int ldo, float* lse, int flags, void* stream) {
  return prefix_fwd_call(dtype, G, P, R, ntiles, tiles, row_first, heads, qkv, ldqkv, out, ldo, lse, flags, stream);
}

static int prefix_bwd_call(int dtype, int grad_dtype, int G, int P, int R, int ntiles, const int* tiles,
                           const int* row_first, int heads, const void* qkv, int ldqkv, const void* ofwd, int ldof,
                           const void* dout, int lddo, const float* lse, void* dqkv, int lddqkv, void* ws,
                           size_t ws_bytes, int flags, void* stream) {
  if (!tiles || !row_first || !qkv || !ofwd || !dout || !lse || !dqkv || !ws) return CLIPK_EINVAL;
  if (flags & ~CLIPK_PREFIX_CLS_GROUP0) return CLIPK_EINVAL;
  if (!prefix_shape_ok(G, P, R, ntiles, heads, lddqkv) || ldqkv < 3 * heads * 64 || lddqkv < 3 * heads * 64 ||
      ldof < heads * 64 || lddo < heads * 64)
    return CLIPK_ESHAPE;
  if (ws_bytes < clipk_attention_prefix_ws_bytes(G, ntiles, heads)) return CLIPK_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  const int c0 = (flags & CLIPK_PREFIX_CLS_GROUP0) ? 1 : 0;
#define CLIPK_PBWD(TT, TGG)                                                                            \
  return prefix_bwd<TT, TGG>(G, P, R, ntiles, tiles, row_first, heads, qkv, ldqkv, ofwd, ldof, dout, lddo, \
                             lse, dqkv, lddqkv, part, st, c0)
  if (dtype == CLIPK_F16 && grad_dtype == CLIPK_BF16) CLIPK_PBWD(f16, bf16);
  if (dtype == CLIPK_F16 && grad_dtype == CLIPK_F16) CLIPK_PBWD(f16, f16);
  if (dtype == CLIPK_BF16 && grad_dtype == CLIPK_BF16) CLIPK_PBWD(bf16, bf16);
  if (dtype == CLIPK_F32 && grad_dtype == CLIPK_F32) CLIPK_PBWD(float, float);
  if (dtype == CLIPK_F32 && grad_dtype == CLIPK_F32S) {
    if (lddqkv % 8) return CLIPK_ESHAPE;  // whole 8-column groups per row
    return prefix_bwd<float, float, true>(G, P, R, ntiles, tiles, row_first, heads, qkv, ldqkv, ofwd, ldof, dout,
                                          lddo, lse, dqkv, lddqkv, part, st, c0);
  }
#undef CLIPK_PBWD
  return CLIPK_EDTYPE;
}

extern "C" int clipk_attention_prefix_bwd(int dtype, int grad_dtype, int G, int P, int R, int ntiles,
                                          const int* tiles, const int* row_first, int heads,
                                          const void* qkv, int ldqkv, const void* ofwd, int ldof,
                                          const void* dout, int lddo, const float* lse, void* dqkv,
                                          int lddqkv, void* ws, size_t ws_bytes, void* stream) {
  return prefix_bwd_call(dtype, grad_dtype, G, P, R, ntiles, tiles, row_first, heads, qkv, ldqkv, ofwd, ldof, dout,
                         lddo, lse, dqkv, lddqkv, ws, ws_bytes, 0, stream);
}

extern "C" int clipk_attention_prefix_bwd_ex(int dtype, int grad_dtype, int G, int P, int R, int ntiles,
                                             const int* tiles, const int* row_first, int heads,
                                             const void* qkv, int ldqkv, const void* ofwd, int ldof,
                                             const void* dout, int lddo, const float* lse, void* dqkv,
                                             int lddqkv, void* ws, size_t ws_bytes, int flags, void* stream) {
  return prefix_bwd_call(dtype, grad_dtype, G, P, R, ntiles, tiles, row_first, heads, qkv, ldqkv, ofwd, ldof, dout,
                         lddo, lse, dqkv, lddqkv, ws, ws_bytes, flags, stream);
}
