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
// (group stride R rows), and attention runs over SEGMENTS:
//     segment 0   : queries = the P prefix rows, keys = themselves (causal);
//     segment 1+c : queries = class c's q_len rows, keys = the P prefix rows (all visible)
//                   followed by its own rows (causal).
// Exactly the reference's math, on ~ (P + sum q_len) / (C * L) of the rows.
//
// seg[2c], seg[2c+1] = (group-relative first row, q_len) of class c; P <= 16, q_len <= 16
// (one 16-row MFMA tile each; the host falls back to the plain layout otherwise).
//
// Work unit: one wave per (group, chunk of kSegChunk segments, head): the prefix K/V of
// (g, h) are loaded once per wave and reused by every segment of the chunk. The backward
// accumulates the prefix rows' dK/dV over the chunk in registers and writes one fp32
// partial per chunk; prefix_kv_reduce sums the chunks in a fixed order (deterministic).
#include <cstdlib>

#include "attn_common.h"

namespace clipk {

constexpr int kFwdBatch = 4, kBwdBatch = 2;  // segments whose loads are issued together
constexpr int kSegChunk = 16;  // VALU kernels; MFMA kernels take the chunk as an argument (<= 16)

// Segments per wave of the MFMA kernels (env CLIPK_PREFIX_FWD_CHUNK / _BWD_CHUNK, read once).
static int chunk_env(const char* name, int def) {
  const char* e = getenv(name);
  const int v = e ? atoi(e) : def;
  return v >= 1 && v <= 16 ? v : def;
}
static int fwd_chunk() { static int c = chunk_env("CLIPK_PREFIX_FWD_CHUNK", 16); return c; }
static int bwd_chunk() { static int c = chunk_env("CLIPK_PREFIX_BWD_CHUNK", 16); return c; }

__device__ __forceinline__ void seg_info(const int* __restrict__ seg, int g, int R, int P, int s,
                                         int& q0, int& qn, int& pre) {
  if (s == 0) {
    q0 = g * R; qn = P; pre = 0;
  } else {
    q0 = g * R + seg[2 * (s - 1)];
    qn = min(seg[2 * (s - 1) + 1], 16);
    pre = P;
  }
}

// The chunk's segment table in one VGPR (lane i holds seg[2*(s_begin-1) + i]), read back
// with v_readlane: no dependent scalar-memory round trip inside the segment loop.
__device__ __forceinline__ int load_seg_table(const int* __restrict__ seg, int C, int s_begin, int lane) {
  const int idx = 2 * (s_begin - 1) + lane;
  return (lane < 32 && idx >= 0 && idx < 2 * C) ? seg[idx] : 0;
}
__device__ __forceinline__ void seg_info_reg(int tab, int g, int R, int P, int s, int s_begin, int& q0,
                                             int& qn, int& pre) {
  if (s == 0) {
    q0 = g * R; qn = P; pre = 0;
  } else {
    const int i = 2 * (s - s_begin);
    q0 = g * R + __builtin_amdgcn_readlane(tab, i);
    qn = min(__builtin_amdgcn_readlane(tab, i + 1), 16);
    pre = P;
  }
}

// Unconditional 16-B load (the caller clamps the row to a valid one) with the value
// zeroed in lanes whose row is past the segment: no exec-masked branch around the load,
// so the compiler can count the loads across the segment loop (vmcnt(N), not vmcnt(0)).
__device__ __forceinline__ s16x8 ld16(const void* p) { return *reinterpret_cast<const s16x8*>(p); }
__device__ __forceinline__ s16x8 sel16(s16x8 v, bool ok) {
  const s16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  return ok ? v : z;
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ------------------------------------------------------------------ forward, MFMA (16-bit)
// Software-pipelined over the chunk's segments: the next segment's Q/K/V fragments are in
// flight while the current one is computed (the per-segment work is too small to hide a
// dependent HBM round trip otherwise).
struct SegRows {
  s16x8 q[2], k[2], v[2];
  int q0, qn, pre;
};

template <typename T>
__global__ __launch_bounds__(256) void attn_prefix_fwd_mfma(int G, int C, int P, int R,
                                                            const int* __restrict__ seg, int H,
                                                            int nchunk, int sc, const T* __restrict__ qkv,
                                                            int ldq, T* __restrict__ out, int ldo,
                                                            float* __restrict__ lse) {
  __shared__ CLIPK_LDS_ALIGN short tiles[4][2][16 * TRS];  // per wave: prefix V, own V
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int wid = blockIdx.x * 4 + w;
  if (wid >= G * nchunk * H) return;  // wave-uniform; no block barriers below
  const int h = wid % H, k = (wid / H) % nchunk, g = wid / (H * nchunk);
  const int W = H * 64;
  short* sVp = tiles[w][0];
  short* sVo = tiles[w][1];

  const int s_begin = k * sc, s_end = min((k + 1) * sc, C + 1);
  const int tab = load_seg_table(seg, C, s_begin, lane);
  auto load = [&](int s, SegRows& f) {
    seg_info_reg(tab, g, R, P, s, s_begin, f.q0, f.qn, f.pre);
    const bool ok = r16 < f.qn;
    const T* qp = qkv + ((size_t)f.q0 + min(r16, f.qn - 1)) * ldq + h * 64;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = 8 * g4 + 32 * kk;
      f.q[kk] = ld16(qp + c);
      f.k[kk] = ld16(qp + W + c);
      f.v[kk] = ld16(qp + 2 * W + c);
    }
    (void)ok;
  };

  // Batches of kFwdBatch segments: all their loads issued up front (unconditional, rows
  // and segment indices clamped), then the bodies; waits are counted inside one loop
  // iteration (a load carried across the back edge gets a vmcnt(0) at the loop head).
  const bool pok = r16 < P;
  const T* pp = qkv + ((size_t)g * R + (pok ? r16 : 0)) * ldq + h * 64;
  s16x8 kp[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int c = 8 * g4 + 32 * kk;
    kp[kk] = ld_row16(pp + W + c, pok);
    *reinterpret_cast<s16x8*>(sVp + r16 * TRS + c) = ld_row16(pp + 2 * W + c, pok);
  }
  auto body = [&](int s, SegRows& cur) {
    const int q0 = cur.q0, qn = cur.qn, pre = cur.pre;
    const bool qok = r16 < qn;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {  // rows past the segment: zero (their loads were clamped)
      cur.q[kk] = sel16(cur.q[kk], qok);
      cur.k[kk] = sel16(cur.k[kk], qok);
      cur.v[kk] = sel16(cur.v[kk], qok);
    }
    lds_fence();  // previous segment's transposed reads of sVo are done
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
      vq[r] = (key <= r16 && key < qn) ? so[r] * kScale : -INFINITY;  // own key 0 always valid
      mx = fmaxf(mx, fmaxf(vp[r], vq[r]));
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float ep[4], eo[4], ps = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ep[r] = __expf(vp[r] - mx);
      eo[r] = __expf(vq[r] - mx);
      ps += ep[r] + eo[r];
    }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    lds_fence();
    // O^T = V^T P^T: the transposed V read doubles as the A operand (A[m=d][k=key]) and the
    // probabilities as B (B[k=key 4g4+jj][n=query r16]), so lane (r16, g4) ends up holding
    // O[query r16][d = 16t + 4g4 .. +3]: one 8-byte store per 16 columns.
    const s16x4 bp = pack4<T>(ep[0], ep[1], ep[2], ep[3]);
    const s16x4 bo = pack4<T>(eo[0], eo[1], eo[2], eo[3]);
    const float inv = 1.0f / ps;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x4 o = mfma16_t<T>(tr_read(sVp, 4 * g4, 16 * t, lane), bp, (f32x4){0.f, 0.f, 0.f, 0.f});
      o = mfma16_t<T>(tr_read(sVo, 4 * g4, 16 * t, lane), bo, o);
      if (qok) store4<T>(out + ((size_t)q0 + r16) * ldo + h * 64 + 16 * t + 4 * g4, o[0] * inv, o[1] * inv,
                         o[2] * inv, o[3] * inv);
    }
    if (lse && g4 == 0 && qok) lse[((size_t)q0 + r16) * H + h] = mx + __logf(ps);
  };
  for (int s = s_begin; s < s_end; s += kFwdBatch) {
    SegRows rr[kFwdBatch];
#pragma unroll
    for (int j = 0; j < kFwdBatch; ++j) load(min(s + j, s_end - 1), rr[j]);
    __builtin_amdgcn_sched_barrier(0);  // every load of the batch issues before the first wait
#pragma unroll
    for (int j = 0; j < kFwdBatch; ++j)
      if (s + j < s_end) body(s + j, rr[j]);
  }
}

// ------------------------------------------------------------------ backward, MFMA (bf16 math)
// Per segment, with the two 16-key tiles (prefix, own) handled like attn_bwd_mfma16:
// S / dP in both accumulator layouts, D_i = rowsum(P o dP) over both tiles in registers,
// dV = P^T dO, dK = dS^T Q, dQ = dS_pre K_pre + dS_own K_own. Pipelined like the forward.
struct SegRowsB {
  s16x8 q[2], k[2], v[2], d[2];
  float l2, l1[4];
  int q0, qn, pre;
};

template <typename T, typename TG>
__global__ __launch_bounds__(256) void attn_prefix_bwd_mfma(int G, int C, int P, int R,
                                                            const int* __restrict__ seg, int H,
                                                            int nchunk, int sc, const T* __restrict__ qkv,
                                                            int ldq, const TG* __restrict__ dout,
                                                            int lddo, const float* __restrict__ lse,
                                                            TG* __restrict__ dqkv, int lddq,
                                                            float* __restrict__ part) {
  static_assert(__is_same(TG, bf16), "MFMA attention backward computes in bf16");
  __shared__ CLIPK_LDS_ALIGN short tiles[4][4][16 * TRS];  // per wave: K_pre, K_own, Q, dO
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int wid = blockIdx.x * 4 + w;
  if (wid >= G * nchunk * H) return;  // wave-uniform
  const int h = wid % H, k = (wid / H) % nchunk, g = wid / (H * nchunk);
  const int W = H * 64;
  short* tKp = tiles[w][0];
  short* tKo = tiles[w][1];
  short* tQ = tiles[w][2];
  short* tD = tiles[w][3];
  const float* lse_h = lse + h;

  const int s_begin = k * sc, s_end = min((k + 1) * sc, C + 1);
  const int tab = load_seg_table(seg, C, s_begin, lane);
  auto load = [&](int s, SegRowsB& f) {
    seg_info_reg(tab, g, R, P, s, s_begin, f.q0, f.qn, f.pre);
    const bool ok = r16 < f.qn;
    const size_t row = (size_t)f.q0 + min(r16, f.qn - 1);
    const T* qp = qkv + row * ldq + h * 64;
    const TG* dp = dout + row * lddo + h * 64;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = 8 * g4 + 32 * kk;
      f.q[kk] = ld16(qp + c);
      f.k[kk] = ld16(qp + W + c);
      f.v[kk] = ld16(qp + 2 * W + c);
      f.d[kk] = ld16(dp + c);
    }
    (void)ok;
    f.l2 = lse_h[row * H];
#pragma unroll
    for (int r = 0; r < 4; ++r) f.l1[r] = lse_h[((size_t)f.q0 + min(4 * g4 + r, f.qn - 1)) * H];
  };

  // batches of kBwdBatch segments, as in the forward
  const bool pok = r16 < P;
  const T* pp = qkv + ((size_t)g * R + (pok ? r16 : 0)) * ldq + h * 64;
  s16x8 kp[2], vp[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int c = 8 * g4 + 32 * kk;
    kp[kk] = to_bf16x8<T>(ld_row16(pp + W + c, pok));
    vp[kk] = to_bf16x8<T>(ld_row16(pp + 2 * W + c, pok));
    *reinterpret_cast<s16x8*>(tKp + r16 * TRS + c) = kp[kk];
  }
  f32x4 dkp[4], dvp[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    dkp[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    dvp[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  auto body = [&](int s, SegRowsB& cur) {
    const int q0 = cur.q0, qn = cur.qn, pre = cur.pre;
    const bool qok = r16 < qn;
    s16x8 q[2], ko[2], vo[2], d[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {  // rows past the segment: zero (their loads were clamped)
      q[kk] = to_bf16x8<T>(sel16(cur.q[kk], qok));
      ko[kk] = to_bf16x8<T>(sel16(cur.k[kk], qok));
      vo[kk] = to_bf16x8<T>(sel16(cur.v[kk], qok));
      d[kk] = sel16(cur.d[kk], qok);
    }
    lds_fence();  // previous segment's transposed reads are done
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
      s1p = mfma32_bf16(q[kk], kp[kk], s1p);   // S  [i=4g4+r][j=r16]
      s2p = mfma32_bf16(kp[kk], q[kk], s2p);   // S^T[j=4g4+r][i=r16]
      p1p = mfma32_bf16(d[kk], vp[kk], p1p);   // dP [i][j]
      p2p = mfma32_bf16(vp[kk], d[kk], p2p);   // dP^T
      s1o = mfma32_bf16(q[kk], ko[kk], s1o);
      s2o = mfma32_bf16(ko[kk], q[kk], s2o);
      p1o = mfma32_bf16(d[kk], vo[kk], p1o);
      p2o = mfma32_bf16(vo[kk], d[kk], p2o);
    }
    // layout 2: i = r16, j = 4g4+r
    const float li2 = cur.l2;
    float P2p[4], P2o[4], Dsum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 4 * g4 + r;
      P2p[r] = (qok && j < pre) ? __expf(s2p[r] * kScale - li2) : 0.f;
      P2o[r] = (qok && j <= r16) ? __expf(s2o[r] * kScale - li2) : 0.f;
      Dsum += P2p[r] * p2p[r] + P2o[r] * p2o[r];
    }
    Dsum += __shfl_xor(Dsum, 16, 64);
    Dsum += __shfl_xor(Dsum, 32, 64);  // D_i for i = r16
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
      const bool iok = i < qn;
      const float li = cur.l1[r];
      const float Di = __shfl(Dsum, i, 64);
      P1p[r] = (iok && r16 < pre) ? __expf(s1p[r] * kScale - li) : 0.f;
      P1o[r] = (iok && r16 <= i) ? __expf(s1o[r] * kScale - li) : 0.f;
      dS1p[r] = P1p[r] * (p1p[r] - Di);
      dS1o[r] = P1o[r] * (p1o[r] - Di);
    }
    // Transposed products (operands swapped), so each lane holds 4 consecutive columns of
    // one row: dV^T = dO^T P, dK^T = Q^T dS, dQ^T = K^T dS^T with the transposed LDS reads
    // as A and the probability / dS registers as B. Lane (r16, g4), tile t: row r16,
    // columns 16t + 4g4 .. +3.
    const s16x4 bPp = pack_bf16x4(P1p[0], P1p[1], P1p[2], P1p[3]);      // B[k=i][n=j]
    const s16x4 bSp = pack_bf16x4(dS1p[0], dS1p[1], dS1p[2], dS1p[3]);
    const s16x4 bPo = pack_bf16x4(P1o[0], P1o[1], P1o[2], P1o[3]);
    const s16x4 bSo = pack_bf16x4(dS1o[0], dS1o[1], dS1o[2], dS1o[3]);
    const s16x4 bTp = pack_bf16x4(dS2p[0], dS2p[1], dS2p[2], dS2p[3]);  // B[k=j][n=i]
    const s16x4 bTo = pack_bf16x4(dS2o[0], dS2o[1], dS2o[2], dS2o[3]);
    lds_fence();
    const bool own_is_prefix = s == 0;  // segment 0's keys are the prefix rows themselves
    TG* orow = dqkv + ((size_t)q0 + r16) * lddq + h * 64 + 4 * g4;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const s16x4 aD = tr_read(tD, 4 * g4, 16 * t, lane);
      const s16x4 aQ = tr_read(tQ, 4 * g4, 16 * t, lane);
      dvp[t] = mfma16_bf16(aD, bPp, dvp[t]);
      dkp[t] = mfma16_bf16(aQ, bSp, dkp[t]);
      f32x4 dq = mfma16_bf16(tr_read(tKp, 4 * g4, 16 * t, lane), bTp, z);
      dq = mfma16_bf16(tr_read(tKo, 4 * g4, 16 * t, lane), bTo, dq);
      const f32x4 dvo = mfma16_bf16(aD, bPo, z);
      const f32x4 dko = mfma16_bf16(aQ, bSo, z);
      if (own_is_prefix) {
        dvp[t] += dvo;
        dkp[t] += dko;
      }
      if (qok) {
        store4<TG>(orow + 16 * t, dq[0] * kScale, dq[1] * kScale, dq[2] * kScale, dq[3] * kScale);
        if (!own_is_prefix) {
          store4<TG>(orow + W + 16 * t, dko[0] * kScale, dko[1] * kScale, dko[2] * kScale, dko[3] * kScale);
          store4<TG>(orow + 2 * W + 16 * t, dvo[0], dvo[1], dvo[2], dvo[3]);
        }
      }
    }
  };
  for (int s = s_begin; s < s_end; s += kBwdBatch) {
    SegRowsB rr[kBwdBatch];
#pragma unroll
    for (int j = 0; j < kBwdBatch; ++j) load(min(s + j, s_end - 1), rr[j]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < kBwdBatch; ++j)
      if (s + j < s_end) body(s + j, rr[j]);
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

// ------------------------------------------------------------------ VALU versions (fp32 path)
// One wave per (group, chunk, head); 4 segments in flight (lane group grp = lane>>4), lane
// r16 = query row (forward, dQ) or key row (dK/dV). K/V rows staged in LDS as fp32.
template <typename T>
__global__ __launch_bounds__(64) void attn_prefix_fwd_valu(int G, int C, int P, int R,
                                                           const int* __restrict__ seg, int H,
                                                           int nchunk, const T* __restrict__ qkv,
                                                           int ldq, T* __restrict__ out, int ldo,
                                                           float* __restrict__ lse) {
  __shared__ CLIPK_LDS_ALIGN float sKp[16 * 64];
  __shared__ CLIPK_LDS_ALIGN float sVp[16 * 64];
  __shared__ CLIPK_LDS_ALIGN float sK[4][16 * 64];
  __shared__ CLIPK_LDS_ALIGN float sV[4][16 * 64];
  const int lane = threadIdx.x, grp = lane >> 4, r16 = lane & 15;
  const int wid = blockIdx.x;
  const int h = wid % H, k = (wid / H) % nchunk, g = wid / (H * nchunk);
  const int W = H * 64;
  {
    const int row = lane >> 2, qtr = lane & 3;  // 16 rows x 4 quarters of 16 values
    float kv[16], vv[16];
    if (row < P) {
      const T* b = qkv + ((size_t)g * R + row) * ldq + h * 64 + qtr * 16;
      constexpr int V = Vec16<T>::N;
#pragma unroll
      for (int c = 0; c < 16 / V; ++c) {
        load16_f32<T>(b + W + c * V, kv + c * V);
        load16_f32<T>(b + 2 * W + c * V, vv + c * V);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c) { kv[c] = 0.f; vv[c] = 0.f; }
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      sKp[row * 64 + qtr * 16 + c] = kv[c];
      sVp[row * 64 + qtr * 16 + c] = vv[c];
    }
  }
  const int s_end = min((k + 1) * kSegChunk, C + 1);
  for (int base = k * kSegChunk; base < s_end; base += 4) {
    const int s = base + grp;
    const bool active = s < s_end;
    int q0 = 0, qn = 0, pre = 0;
    if (active) seg_info(seg, g, R, P, s, q0, qn, pre);
    const bool qok = active && r16 < qn;
    const T* qp = qkv + ((size_t)q0 + (qok ? r16 : 0)) * ldq + h * 64;
    float q[64], t64[64];
    load_row64<T>(qp, q);
#pragma unroll
    for (int dd = 0; dd < 64; ++dd) q[dd] *= kScale;
    load_row64<T>(qp + W, t64);
#pragma unroll
    for (int dd = 0; dd < 64; ++dd) sK[grp][r16 * 64 + dd] = t64[dd];
    load_row64<T>(qp + 2 * W, t64);
#pragma unroll
    for (int dd = 0; dd < 64; ++dd) sV[grp][r16 * 64 + dd] = t64[dd];
    __syncthreads();
    float sc[32], m = -INFINITY;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      sc[j] = j < pre ? dot64(q, &sKp[j * 64]) : -INFINITY;
      sc[16 + j] = (j <= r16 && j < qn) ? dot64(q, &sK[grp][j * 64]) : -INFINITY;
      m = fmaxf(m, fmaxf(sc[j], sc[16 + j]));
    }
    float l = 0.f;
#pragma unroll
    for (int dd = 0; dd < 64; ++dd) t64[dd] = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      if (sc[j] != -INFINITY) {
        const float p = __expf(sc[j] - m);
        l += p;
        const float* vr = j < 16 ? &sVp[j * 64] : &sV[grp][(j - 16) * 64];
#pragma unroll
        for (int dd = 0; dd < 64; ++dd) t64[dd] = fmaf(p, vr[dd], t64[dd]);
      }
    }
    if (qok) {
      const float inv = 1.0f / l;
#pragma unroll
      for (int dd = 0; dd < 64; ++dd) t64[dd] *= inv;
      store_row64<T>(out + ((size_t)q0 + r16) * ldo + h * 64, t64);
      if (lse) lse[((size_t)q0 + r16) * H + h] = m + __logf(l);
    }
    __syncthreads();  // sK/sV reused by the next 4 segments
  }
}

template <typename T, typename TG>
__global__ __launch_bounds__(64) void attn_prefix_bwd_valu(
    int G, int C, int P, int R, const int* __restrict__ seg, int H, int nchunk,
    const T* __restrict__ qkv, int ldq, const T* __restrict__ o_fwd, int ldof,
    const TG* __restrict__ dout, int lddo, const float* __restrict__ lse, TG* __restrict__ dqkv,
    int lddq, float* __restrict__ part) {
  __shared__ CLIPK_LDS_ALIGN float sKp[16 * 64];
  __shared__ CLIPK_LDS_ALIGN float sVp[16 * 64];
  __shared__ CLIPK_LDS_ALIGN float sQ[4][16 * 64];   // scaled q
  __shared__ CLIPK_LDS_ALIGN float sK[4][16 * 64];
  __shared__ CLIPK_LDS_ALIGN float sV[4][16 * 64];
  __shared__ CLIPK_LDS_ALIGN float sdO[4][16 * 64];
  __shared__ CLIPK_LDS_ALIGN float sAk[4][16 * 64];  // prefix dK accumulators, per lane group
  __shared__ CLIPK_LDS_ALIGN float sAv[4][16 * 64];
  __shared__ float slse[4][16], sD[4][16];
  const int lane = threadIdx.x, grp = lane >> 4, r16 = lane & 15;
  const int wid = blockIdx.x;
  const int h = wid % H, k = (wid / H) % nchunk, g = wid / (H * nchunk);
  const int W = H * 64;
  {
    const int row = lane >> 2, qtr = lane & 3;
    float kv[16], vv[16];
    if (row < P) {
      const T* b = qkv + ((size_t)g * R + row) * ldq + h * 64 + qtr * 16;
      constexpr int V = Vec16<T>::N;
#pragma unroll
      for (int c = 0; c < 16 / V; ++c) {
        load16_f32<T>(b + W + c * V, kv + c * V);
        load16_f32<T>(b + 2 * W + c * V, vv + c * V);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c) { kv[c] = 0.f; vv[c] = 0.f; }
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      sKp[row * 64 + qtr * 16 + c] = kv[c];
      sVp[row * 64 + qtr * 16 + c] = vv[c];
    }
  }
  for (int i = lane; i < 4 * 16 * 64; i += 64) {
    (&sAk[0][0])[i] = 0.f;
    (&sAv[0][0])[i] = 0.f;
  }
  const int s_end = min((k + 1) * kSegChunk, C + 1);
  for (int base = k * kSegChunk; base < s_end; base += 4) {
    const int s = base + grp;
    const bool active = s < s_end;
    int q0 = 0, qn = 0, pre = 0;
    if (active) seg_info(seg, g, R, P, s, q0, qn, pre);
    const bool qok = active && r16 < qn;
    const size_t row = (size_t)q0 + (qok ? r16 : 0);
    const T* qp = qkv + row * ldq + h * 64;
    float a[64], dO[64];
    load_row64<T>(qp, a);
#pragma unroll
    for (int dd = 0; dd < 64; ++dd) sQ[grp][r16 * 64 + dd] = a[dd] * kScale;
    load_row64<T>(qp + W, a);
#pragma unroll
    for (int dd = 0; dd < 64; ++dd) sK[grp][r16 * 64 + dd] = a[dd];
    load_row64<T>(qp + 2 * W, a);
#pragma unroll
    for (int dd = 0; dd < 64; ++dd) sV[grp][r16 * 64 + dd] = a[dd];
    load_row64<TG>(dout + row * lddo + h * 64, dO);
    load_row64<T>(o_fwd + row * ldof + h * 64, a);
    const float Di = qok ? dot64(dO, a) : 0.f;
#pragma unroll
    for (int dd = 0; dd < 64; ++dd) sdO[grp][r16 * 64 + dd] = qok ? dO[dd] : 0.f;
    const float li = qok ? lse[row * H + h] : 0.f;
    slse[grp][r16] = li;
    sD[grp][r16] = Di;
    __syncthreads();
    // phase 1 (lane = query): dq = sum_j P (dP - D) k_j / 8 over prefix + own keys
    {
      const float* qi = &sQ[grp][r16 * 64];
#pragma unroll
      for (int dd = 0; dd < 64; ++dd) a[dd] = 0.f;
      for (int j = 0; j < 32; ++j) {
        const bool ok = j < 16 ? j < pre : (j - 16 <= r16 && j - 16 < qn);
        if (!qok || !ok) continue;
        const float* kr = j < 16 ? &sKp[j * 64] : &sK[grp][(j - 16) * 64];
        const float* vr = j < 16 ? &sVp[j * 64] : &sV[grp][(j - 16) * 64];
        const float p = __expf(dot64(qi, kr) - li);
        const float ds = p * (dot64(dO, vr) - Di);
#pragma unroll
        for (int dd = 0; dd < 64; ++dd) a[dd] = fmaf(ds, kr[dd], a[dd]);
      }
      if (qok) {
#pragma unroll
        for (int dd = 0; dd < 64; ++dd) a[dd] *= kScale;
        store_row64<TG>(dqkv + row * lddq + h * 64, a);
      }
    }
    // phase 2 (lane = own key j = r16): over queries i >= j of this segment
    {
      const float* kj = &sK[grp][r16 * 64];
      const float* vj = &sV[grp][r16 * 64];
      float dk[64], dv[64];
#pragma unroll
      for (int dd = 0; dd < 64; ++dd) { dk[dd] = 0.f; dv[dd] = 0.f; }
      for (int i = r16; i < qn; ++i) {
        const float* qr = &sQ[grp][i * 64];
        const float* dr = &sdO[grp][i * 64];
        const float p = __expf(dot64(qr, kj) - slse[grp][i]);
        const float ds = p * (dot64(dr, vj) - sD[grp][i]);
#pragma unroll
        for (int dd = 0; dd < 64; ++dd) {
          dv[dd] = fmaf(p, dr[dd], dv[dd]);
          dk[dd] = fmaf(ds, qr[dd], dk[dd]);
        }
      }
      if (qok) {
        if (s == 0) {  // segment 0's own keys are the prefix rows: accumulate
#pragma unroll
          for (int dd = 0; dd < 64; ++dd) {
            sAk[grp][r16 * 64 + dd] += dk[dd];
            sAv[grp][r16 * 64 + dd] += dv[dd];
          }
        } else {
          store_row64<TG>(dqkv + row * lddq + W + h * 64, dk);
          store_row64<TG>(dqkv + row * lddq + 2 * W + h * 64, dv);
        }
      }
    }
    // phase 3 (lane = prefix key j = r16): partial over every query of this segment
    if (active && r16 < pre) {
      const float* kj = &sKp[r16 * 64];
      const float* vj = &sVp[r16 * 64];
      float dk[64], dv[64];
#pragma unroll
      for (int dd = 0; dd < 64; ++dd) { dk[dd] = 0.f; dv[dd] = 0.f; }
      for (int i = 0; i < qn; ++i) {
        const float* qr = &sQ[grp][i * 64];
        const float* dr = &sdO[grp][i * 64];
        const float p = __expf(dot64(qr, kj) - slse[grp][i]);
        const float ds = p * (dot64(dr, vj) - sD[grp][i]);
#pragma unroll
        for (int dd = 0; dd < 64; ++dd) {
          dv[dd] = fmaf(p, dr[dd], dv[dd]);
          dk[dd] = fmaf(ds, qr[dd], dk[dd]);
        }
      }
#pragma unroll
      for (int dd = 0; dd < 64; ++dd) {
        sAk[grp][r16 * 64 + dd] += dk[dd];
        sAv[grp][r16 * 64 + dd] += dv[dd];
      }
    }
    __syncthreads();  // staging buffers reused by the next 4 segments
  }
  float* pb = part + ((size_t)g * nchunk + k) * 16 * (2 * W);
  for (int idx = lane; idx < P * 64; idx += 64) {
    const int j = idx >> 6, dd = idx & 63;
    const int o = j * 64 + dd;
    pb[(size_t)j * 2 * W + h * 64 + dd] = ((sAk[0][o] + sAk[1][o]) + sAk[2][o]) + sAk[3][o];
    pb[(size_t)j * 2 * W + W + h * 64 + dd] = ((sAv[0][o] + sAv[1][o]) + sAv[2][o]) + sAv[3][o];
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
  float acc = 0.f;
  for (int k = 0; k < nchunk; ++k) acc += src[(size_t)k * 16 * 2 * W];
  dqkv[((size_t)g * R + p) * lddq + W + col] = (TG)acc;
}

static inline int n_chunks(int C, int sc = kSegChunk) { return (C + 1 + sc - 1) / sc; }

template <typename T>
static int prefix_fwd(int G, int C, int P, int R, const int* seg, int H, const void* qkv, int ldq,
                      void* out, int ldo, float* lse, hipStream_t st) {
  if constexpr (sizeof(T) == 2) {
    const int sc = fwd_chunk();
    const int nchunk = n_chunks(C, sc);
    const long waves = (long)G * nchunk * H;
    hipLaunchKernelGGL((attn_prefix_fwd_mfma<T>), dim3((waves + 3) / 4), dim3(256), 0, st, G, C, P, R, seg,
                       H, nchunk, sc, (const T*)qkv, ldq, (T*)out, ldo, lse);
  } else {
    const int nchunk = n_chunks(C);
    const long waves = (long)G * nchunk * H;
    hipLaunchKernelGGL((attn_prefix_fwd_valu<T>), dim3(waves), dim3(64), 0, st, G, C, P, R, seg, H, nchunk,
                       (const T*)qkv, ldq, (T*)out, ldo, lse);
  }
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

template <typename T, typename TG>
static int prefix_bwd(int G, int C, int P, int R, const int* seg, int H, const void* qkv, int ldq,
                      const void* ofwd, int ldof, const void* dout, int lddo, const float* lse,
                      void* dqkv, int lddq, float* part, hipStream_t st) {
  constexpr bool mfma = __is_same(TG, bf16) && sizeof(T) == 2;
  const int sc = mfma ? bwd_chunk() : kSegChunk;
  const int nchunk = n_chunks(C, sc);
  const long waves = (long)G * nchunk * H;
  if constexpr (mfma) {
    hipLaunchKernelGGL((attn_prefix_bwd_mfma<T, TG>), dim3((waves + 3) / 4), dim3(256), 0, st, G, C, P, R,
                       seg, H, nchunk, sc, (const T*)qkv, ldq, (const TG*)dout, lddo, lse, (TG*)dqkv, lddq,
                       part);
  } else {
    hipLaunchKernelGGL((attn_prefix_bwd_valu<T, TG>), dim3(waves), dim3(64), 0, st, G, C, P, R, seg, H,
                       nchunk, (const T*)qkv, ldq, (const T*)ofwd, ldof, (const TG*)dout, lddo, lse,
                       (TG*)dqkv, lddq, part);
  }
  CLIPK_CHECK_LAUNCH();
  const int W = H * 64;
  hipLaunchKernelGGL((prefix_kv_reduce<TG>), dim3(G * P, (2 * W + 255) / 256), dim3(256), 0, st, P, R, W,
                     nchunk, part, (TG*)dqkv, lddq);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

}  // namespace clipk

using namespace clipk;

static int prefix_shape_ok(int G, int C, int P, int R, int max_q, int heads) {
  return G > 0 && C > 0 && P >= 1 && P <= 16 && max_q >= 1 && max_q <= 16 && R >= P + C && heads > 0;
}

extern "C" size_t clipk_attention_prefix_ws_bytes(int G, int C, int heads) {
  if (G <= 0 || C <= 0 || heads <= 0) return 0;
  const int sc = bwd_chunk() < kSegChunk ? bwd_chunk() : kSegChunk;  // the larger chunk count of the two paths
  return (size_t)G * n_chunks(C, sc) * 16 * 2 * heads * 64 * sizeof(float);
}

extern "C" int clipk_attention_prefix_fwd(int dtype, int G, int C, int P, int R, const int* seg,
                                          int max_q, int heads, const void* qkv, int ldqkv,
                                          void* out, int ldo, float* lse, void* stream) {
  if (!seg || !qkv || !out) return CLIPK_EINVAL;
  if (!prefix_shape_ok(G, C, P, R, max_q, heads) || ldqkv < 3 * heads * 64 || ldo < heads * 64 ||
      ldqkv % 8 || ldo % 8)
    return CLIPK_ESHAPE;
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case CLIPK_F16: return prefix_fwd<f16>(G, C, P, R, seg, heads, qkv, ldqkv, out, ldo, lse, st);
    case CLIPK_BF16: return prefix_fwd<bf16>(G, C, P, R, seg, heads, qkv, ldqkv, out, ldo, lse, st);
    case CLIPK_F32: return prefix_fwd<float>(G, C, P, R, seg, heads, qkv, ldqkv, out, ldo, lse, st);
    default: return CLIPK_EDTYPE;
  }
}

extern "C" int clipk_attention_prefix_bwd(int dtype, int grad_dtype, int G, int C, int P, int R,
                                          const int* seg, int max_q, int heads, const void* qkv,
                                          int ldqkv, const void* ofwd, int ldof, const void* dout,
                                          int lddo, const float* lse, void* dqkv, int lddqkv,
                                          void* ws, size_t ws_bytes, void* stream) {
  if (!seg || !qkv || !ofwd || !dout || !lse || !dqkv || !ws) return CLIPK_EINVAL;
  if (!prefix_shape_ok(G, C, P, R, max_q, heads) || ldqkv < 3 * heads * 64 ||
      lddqkv < 3 * heads * 64 || ldof < heads * 64 || lddo < heads * 64)
    return CLIPK_ESHAPE;
  if (ws_bytes < clipk_attention_prefix_ws_bytes(G, C, heads)) return CLIPK_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
#define CLIPK_PBWD(TT, TGG)                                                                      \
  return prefix_bwd<TT, TGG>(G, C, P, R, seg, heads, qkv, ldqkv, ofwd, ldof, dout, lddo, lse, dqkv, \
                             lddqkv, part, st)
  if (dtype == CLIPK_F16 && grad_dtype == CLIPK_BF16) CLIPK_PBWD(f16, bf16);
  if (dtype == CLIPK_F16 && grad_dtype == CLIPK_F16) CLIPK_PBWD(f16, f16);
  if (dtype == CLIPK_BF16 && grad_dtype == CLIPK_BF16) CLIPK_PBWD(bf16, bf16);
  if (dtype == CLIPK_F32 && grad_dtype == CLIPK_F32) CLIPK_PBWD(float, float);
#undef CLIPK_PBWD
  return CLIPK_EDTYPE;
}
