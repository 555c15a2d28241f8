// Multi-head self-attention core (head dim 64) for CLIP's nn.MultiheadAttention
// (PromptSRC/clip/model.py:171,181-183): softmax(q k^T / 8 + mask) v with the causal
// -inf-above-diagonal text mask (model.py:592-598) or no mask (vision).
//
// Input is the packed in_proj output row [(s*L+t), 3*W] (q | k | v, head h at columns
// h*64 of each third), exactly what the QKV GEMM writes, so no reshuffle pass exists.
//
// Short sequences (text, L <= 64 after EOT truncation): G = 64/LP (seq, head) pairs per
// wave, lane = query row; the pair's K/V rows staged once in LDS and read back as
// 16-B broadcasts; scores for the whole row kept in registers (fully unrolled over LP);
// exact two-pass softmax. Long sequences (vision, L up to 577): 256 query rows per
// block, keys streamed through LDS in chunks of 64 with an online softmax.
// Backward (text): lane = query row for dQ, lane = key row for dK/dV, recomputing
// P from the saved log-sum-exp; D_i = dO_i . O_i from the saved forward output.
#include "attn_common.h"

namespace clipk {

// ------------------------------------------------------------------ forward, L <= LP <= 64
template <int LP, typename T>
__global__ __launch_bounds__(256) void attn_fwd_short(int nseq, int L, int H, int causal,
                                                      const T* __restrict__ qkv, int ldq,
                                                      T* __restrict__ out, int ldo,
                                                      float* __restrict__ lse) {
  constexpr int G = 64 / LP;
  constexpr int V = Vec16<T>::N;
  // per wave: G*LP = 64 rows of K then 64 rows of V, 64 elements each
  __shared__ CLIPK_LDS_ALIGN T sk[4][64 * 64];
  __shared__ CLIPK_LDS_ALIGN T sv[4][64 * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane / LP, i = lane % LP;
  const int pair = (blockIdx.x * 4 + w) * G + g;
  const bool pair_ok = pair < nseq * H;
  const int s = pair_ok ? pair / H : 0, h = pair_ok ? pair % H : 0;
  const int W = H * 64;
  const bool row_ok = pair_ok && i < L;
  const size_t row = (size_t)s * L + (row_ok ? i : 0);
  const T* qp = qkv + row * ldq + h * 64;

  // stage own K/V rows
  T* myk = &sk[w][lane * 64];
  T* myv = &sv[w][lane * 64];
  if (row_ok) {
#pragma unroll
    for (int c = 0; c < 64 / V; ++c) {
      *reinterpret_cast<u32x4*>(myk + c * V) =
          *reinterpret_cast<const u32x4*>(qp + W + c * V);
      *reinterpret_cast<u32x4*>(myv + c * V) =
          *reinterpret_cast<const u32x4*>(qp + 2 * W + c * V);
    }
  }
  float q[64];
  load_row64<T>(qp, q);
#pragma unroll
  for (int d = 0; d < 64; ++d) q[d] *= kScale;
  __syncthreads();

  const T* gk = &sk[w][g * LP * 64];
  const T* gv = &sv[w][g * LP * 64];
  float sc[LP];
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < LP; ++j) {
    if (j < L) {
      float kr[64];
      load_row64<T>(gk + j * 64, kr);
      float v = dot64(q, kr);
      if (causal && j > i) v = -INFINITY;
      sc[j] = v;
      m = fmaxf(m, v);
    } else {
      sc[j] = -INFINITY;
    }
  }
  float l = 0.f;
  float o[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) o[d] = 0.f;
#pragma unroll
  for (int j = 0; j < LP; ++j) {
    if (j < L) {
      const float p = __expf(sc[j] - m);
      l += p;
      float vr[64];
      load_row64<T>(gv + j * 64, vr);
#pragma unroll
      for (int d = 0; d < 64; ++d) o[d] = fmaf(p, vr[d], o[d]);
    }
  }
  if (row_ok) {
    const float inv = 1.0f / l;
#pragma unroll
    for (int d = 0; d < 64; ++d) o[d] *= inv;
    store_row64<T>(out + row * ldo + h * 64, o);
    if (lse) lse[row * H + h] = m + __logf(l);
  }
}

// ------------------------------------------------------------------ forward, any L, fp32
// (PREC fp32 / fp32s: the ViT's L = 50..577, plain text 64 < L <= 77). Block = 64 query rows of
// one (sequence, head), 4 waves of 16 rows; lane = 4 r + s holds row r's 16-column slice s of q
// and o (the interleaved map of attn_common.h); K / V in 64-key LDS chunks, a score is 16 FMAs
// + a quad sum, exact online softmax.
__global__ __launch_bounds__(256) void attn_fwd_f32(int nseq, int L, int H, int causal, const float* __restrict__ qkv,
                                                    int ldq, float* __restrict__ out, int ldo,
                                                    float* __restrict__ lse) {
  __shared__ CLIPK_LDS_ALIGN float sk[64 * 64];
  __shared__ CLIPK_LDS_ALIGN float sv[64 * 64];
  const int tid = threadIdx.x, lane = tid & 63, r = lane >> 2, s = lane & 3;
  const int h = blockIdx.y, sq = blockIdx.z;
  const int W = H * 64;
  const int i = blockIdx.x * 64 + (tid >> 6) * 16 + r;  // query row
  const bool row_ok = i < L;
  const size_t row = (size_t)sq * L + (row_ok ? i : L - 1);
  float q[16], o[16];
  ld16x(qkv + row * ldq + h * 64 + kSl * s, q);
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    q[d] *= kScale;
    o[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  const int qmax = min(L, (int)(blockIdx.x + 1) * 64) - 1;
  const int jend = causal ? qmax + 1 : L;
  for (int j0 = 0; j0 < jend; j0 += 64) {
    __syncthreads();
    {  // 64 key / value rows: thread -> (row tid / 4, 16-column quarter)
      const int jr = j0 + (tid >> 2), part = tid & 3;
      float t[16];
      if (jr < L) {
        const float* base = qkv + ((size_t)sq * L + jr) * ldq + h * 64 + part * kSl;
        ld16x(base + W, t);
        st16x(&sk[(tid >> 2) * 64 + part * kSl], t);
        ld16x(base + 2 * W, t);
        st16x(&sv[(tid >> 2) * 64 + part * kSl], t);
      }
    }
    __syncthreads();
    const int nj = min(64, jend - j0);
    for (int j = 0; j < nj; ++j) {
      float kv[16];
      ld16x(&sk[j * 64 + kSl * s], kv);
      const float sc = quad_sum(dot16(q, kv));
      if (!causal || j0 + j <= i) {
        if (sc > m) {
          const float a = __expf(m - sc);  // 0 for the first key (m = -inf)
          l *= a;
#pragma unroll
          for (int d = 0; d < 16; ++d) o[d] *= a;
          m = sc;
        }
        const float p = __expf(sc - m);
        l += p;
        ld16x(&sv[j * 64 + kSl * s], kv);
#pragma unroll
        for (int d = 0; d < 16; ++d) o[d] = fmaf(p, kv[d], o[d]);
      }
    }
  }
  if (row_ok) {
    const float inv = 1.0f / l;
#pragma unroll
    for (int d = 0; d < 16; ++d) o[d] *= inv;
    st16x(out + row * ldo + h * 64 + kSl * s, o);
    if (lse && s == 0) lse[row * H + h] = m + __logf(l);
  }
}

// ------------------------------------------------------------------ backward, L <= LP <= 64
// qkv/out in T (forward dtype), dout/dqkv in TG (grad dtype).
template <int LP, typename T, typename TG>
__global__ __launch_bounds__(64) void attn_bwd_short(int nseq, int L, int H, int causal,
                                                     const T* __restrict__ qkv, int ldq,
                                                     const T* __restrict__ o_fwd, int ldof,
                                                     const TG* __restrict__ dout, int lddo,
                                                     const float* __restrict__ lse,
                                                     TG* __restrict__ dqkv, int lddq) {
  constexpr int G = 64 / LP;
  __shared__ CLIPK_LDS_ALIGN float sq[64 * 64];   // scaled q rows, later reused
  __shared__ CLIPK_LDS_ALIGN float sk[64 * 64];
  __shared__ CLIPK_LDS_ALIGN float sv[64 * 64];
  __shared__ CLIPK_LDS_ALIGN float sdo[64 * 64];
  __shared__ float slse[64], sD[64];
  const int lane = threadIdx.x;
  const int g = lane / LP, i = lane % LP;
  const int pair = blockIdx.x * G + g;
  const bool pair_ok = pair < nseq * H;
  const int s = pair_ok ? pair / H : 0, h = pair_ok ? pair % H : 0;
  const int W = H * 64;
  const bool row_ok = pair_ok && i < L;
  const size_t row = (size_t)s * L + (row_ok ? i : 0);

  float a[64], b[64];
  // q (scaled) -> LDS, k -> LDS
  load_row64<T>(qkv + row * ldq + h * 64, a);
#pragma unroll
  for (int d = 0; d < 64; ++d) a[d] *= kScale;
  load_row64<T>(qkv + row * ldq + W + h * 64, b);
#pragma unroll
  for (int d = 0; d < 64; d += 4) {
    *reinterpret_cast<f32x4*>(&sq[lane * 64 + d]) = (f32x4){a[d], a[d + 1], a[d + 2], a[d + 3]};
    *reinterpret_cast<f32x4*>(&sk[lane * 64 + d]) = (f32x4){b[d], b[d + 1], b[d + 2], b[d + 3]};
  }
  // v -> LDS ; dO and D_i = dO_i . O_i
  load_row64<T>(qkv + row * ldq + 2 * W + h * 64, b);
#pragma unroll
  for (int d = 0; d < 64; d += 4)
    *reinterpret_cast<f32x4*>(&sv[lane * 64 + d]) = (f32x4){b[d], b[d + 1], b[d + 2], b[d + 3]};
  float dO[64];
  load_row64<TG>(dout + row * lddo + h * 64, dO);
  load_row64<T>(o_fwd + row * ldof + h * 64, b);
  const float Di = dot64(dO, b);
#pragma unroll
  for (int d = 0; d < 64; d += 4)
    *reinterpret_cast<f32x4*>(&sdo[lane * 64 + d]) = (f32x4){dO[d], dO[d + 1], dO[d + 2], dO[d + 3]};
  const float li = row_ok ? lse[row * H + h] : 0.f;
  slse[lane] = li;
  sD[lane] = Di;
  __syncthreads();

  // ---- phase 1: lane = query row i:  dq_i = sum_j P_ij (dP_ij - D_i) k_j / 8
  const float* gq = &sq[g * LP * 64];
  const float* gk = &sk[g * LP * 64];
  const float* gv = &sv[g * LP * 64];
  const float* gdo = &sdo[g * LP * 64];
#pragma unroll
  for (int d = 0; d < 64; ++d) b[d] = 0.f;  // dq accumulator
  const float* qi = &sq[lane * 64];
#pragma unroll
  for (int j = 0; j < LP; ++j) {
    if (j < L && !(causal && j > i)) {
      const float p = __expf(dot64(qi, gk + j * 64) - li);
      const float dp = dot64(dO, gv + j * 64);
      const float ds = p * (dp - Di);
      const float* kr = gk + j * 64;
#pragma unroll
      for (int d = 0; d < 64; ++d) b[d] = fmaf(ds, kr[d], b[d]);
    }
  }
  if (row_ok) {
#pragma unroll
    for (int d = 0; d < 64; ++d) b[d] *= kScale;
    store_row64<TG>(dqkv + row * lddq + h * 64, b);
  }

  // ---- phase 2: lane = key row j:  dv_j = sum_i P_ij dO_i ; dk_j = sum_i dS_ij q_i(scaled)
  const int j = i;
  const float* kj = &sk[lane * 64];
  const float* vj = &sv[lane * 64];
  float dv[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) { dv[d] = 0.f; a[d] = 0.f; }  // a = dk accumulator
  const float* glse = &slse[g * LP];
  const float* gD = &sD[g * LP];
#pragma unroll
  for (int ii = 0; ii < LP; ++ii) {
    if (ii < L && !(causal && j > ii)) {
      const float* qr = gq + ii * 64;
      const float* dor = gdo + ii * 64;
      const float p = __expf(dot64(qr, kj) - glse[ii]);
      const float dp = dot64(dor, vj);
      const float ds = p * (dp - gD[ii]);
#pragma unroll
      for (int d = 0; d < 64; ++d) {
        dv[d] = fmaf(p, dor[d], dv[d]);
        a[d] = fmaf(ds, qr[d], a[d]);
      }
    }
  }
  if (row_ok) {
    store_row64<TG>(dqkv + row * lddq + W + h * 64, a);
    store_row64<TG>(dqkv + row * lddq + 2 * W + h * 64, dv);
  }
}

// ------------------------------------------------------------------ backward, L <= 16, MFMA
// One wave per (seq, head); 16x16 tiles (rows >= L zero-padded and masked).
// S = Q K^T and S^T = K Q^T (and dP, dP^T) with v_mfma_f32_16x16x32; the score
// accumulators are reused in registers as operands of the 16x16x16 products
// (accumulator layout [4*(l>>4)+r][l&15] == the 16x16x16 B layout == transposed A layout):
//   dV = P^T dO, dK = dS^T Q (layout-1 P/dS as A),  dQ = dS K (layout-2 dS as A);
// the row-major dO/Q/K tiles feed those products through ds_read_b64_tr_b16 (hardware
// transposed LDS read). D_i = rowsum(P o dP) is formed in registers (no saved O needed).
// Backward math is bf16 x bf16 -> fp32 (the grad dtype); T is the forward operand type.
template <typename T, typename TG>
__global__ __launch_bounds__(256) void attn_bwd_mfma16(int nseq, int L, int H, int causal,
                                                       const T* __restrict__ qkv, int ldq,
                                                       const TG* __restrict__ dout, int lddo,
                                                       const float* __restrict__ lse,
                                                       TG* __restrict__ dqkv, int lddq) {
  static_assert(sizeof(T) == 2 && sizeof(TG) == 2, "MFMA attention backward: 16-bit operands, math in TG");
  __shared__ CLIPK_LDS_ALIGN short tiles[4][3][16 * TRS];  // per wave: Q, K, dO (bf16)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int pair = blockIdx.x * 4 + w;
  if (pair >= nseq * H) return;  // wave-uniform
  const int s = pair / H, h = pair % H;
  const int W = H * 64;
  const size_t row0 = (size_t)s * L;
  short* tQ = tiles[w][0];
  short* tK = tiles[w][1];
  short* tD = tiles[w][2];

  // ---- fragments: row r16, 16-B chunk g4 (+4 for kk=1) of Q, K, V (T) and dO (TG)
  const bool rok = r16 < L;
  const T* qrow = qkv + (row0 + (rok ? r16 : 0)) * ldq + h * 64;
  const TG* drow = dout + (row0 + (rok ? r16 : 0)) * lddo + h * 64;
  s16x8 q[2], k[2], v[2], d[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int c = 8 * g4 + 32 * kk;
    q[kk] = ld_row16(qrow + c, rok);
    k[kk] = ld_row16(qrow + W + c, rok);
    v[kk] = ld_row16(qrow + 2 * W + c, rok);
    d[kk] = ld_row16(drow + c, rok);
  }
  // stage Q, K, dO (bf16) for the transposed reads
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int c = 8 * g4 + 32 * kk;
    const s16x8 qb = to_g8<T, TG>(q[kk]), kb = to_g8<T, TG>(k[kk]);
    *reinterpret_cast<s16x8*>(tQ + r16 * TRS + c) = qb;
    *reinterpret_cast<s16x8*>(tK + r16 * TRS + c) = kb;
    *reinterpret_cast<s16x8*>(tD + r16 * TRS + c) = d[kk];
    v[kk] = to_g8<T, TG>(v[kk]);
    q[kk] = qb;
    k[kk] = kb;
  }
  // ---- scores in both layouts
  f32x4 s1 = {0, 0, 0, 0}, s2 = {0, 0, 0, 0}, p1 = {0, 0, 0, 0}, p2 = {0, 0, 0, 0};
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    s1 = mfma32_t<TG>(q[kk], k[kk], s1);  // S  [i=4g4+r][j=r16]
    s2 = mfma32_t<TG>(k[kk], q[kk], s2);  // S^T[j=4g4+r][i=r16]
    p1 = mfma32_t<TG>(d[kk], v[kk], p1);  // dP [i][j]
    p2 = mfma32_t<TG>(v[kk], d[kk], p2);  // dP^T
  }
  // ---- layout 2 (i = r16, j = 4g4+r): P, D_i, dS
  const float* lse_h = lse + h;
  const float li2 = rok ? lse_h[(row0 + r16) * H] : 0.f;
  float P2[4], dS2[4], Dsum = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = r16, j = 4 * g4 + r;
    const bool ok = i < L && j < L && !(causal && j > i);
    P2[r] = ok ? __expf(s2[r] * kScale - li2) : 0.f;
    Dsum += P2[r] * p2[r];
  }
  Dsum += __shfl_xor(Dsum, 16, 64);
  Dsum += __shfl_xor(Dsum, 32, 64);  // D_i for i = r16, in every lane of that column
#pragma unroll
  for (int r = 0; r < 4; ++r) dS2[r] = P2[r] * (p2[r] - Dsum);
  // ---- layout 1 (i = 4g4+r, j = r16)
  float P1[4], dS1[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 4 * g4 + r, j = r16;
    const bool ok = i < L && j < L && !(causal && j > i);
    const float li = ok ? lse_h[(row0 + i) * H] : 0.f;
    const float Di = __shfl(Dsum, i, 64);
    P1[r] = ok ? __expf(s1[r] * kScale - li) : 0.f;
    dS1[r] = P1[r] * (p1[r] - Di);
  }
  const s16x4 aP = pack4<TG>(P1[0], P1[1], P1[2], P1[3]);     // A[m=j][k=i] = P[i][j]
  const s16x4 aS = pack4<TG>(dS1[0], dS1[1], dS1[2], dS1[3]); // A[m=j][k=i] = dS[i][j]
  const s16x4 aT = pack4<TG>(dS2[0], dS2[1], dS2[2], dS2[3]); // A[m=i][k=j] = dS[i][j]
  // the tiles are wave-private: LDS ops of one wave complete in order; this wait also
  // fences the compiler (no __syncthreads: waves of a partial block exit early above)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  TG* out = dqkv + h * 64;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f32x4 z = {0, 0, 0, 0};
    const f32x4 dv = mfma16_t<TG>(aP, tr_read(tD, 4 * g4, 16 * t, lane), z);  // [j][d]
    const f32x4 dk = mfma16_t<TG>(aS, tr_read(tQ, 4 * g4, 16 * t, lane), z);  // [j][d]
    const f32x4 dq = mfma16_t<TG>(aT, tr_read(tK, 4 * g4, 16 * t, lane), z);  // [i][d]
    const int col = 16 * t + r16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * g4 + r;
      if (row < L) {
        TG* o = out + (row0 + row) * lddq + col;
        o[0] = (TG)(dq[r] * kScale);
        o[W] = (TG)(dk[r] * kScale);
        o[2 * W] = (TG)dv[r];
      }
    }
  }
}

// ------------------------------------------------------------------ forward, MFMA (any L)
// Flash-style forward on MFMA for 16-bit operands: block = 4 waves = 64 query rows of one
// (seq, head); keys streamed through LDS in chunks of 64 (K and V tiles, row-major); per 32
// keys S^T = K Q^T (16x16x32: query on the lane, 8 keys per lane in registers). Built for low
// VALU per key (the first form -- O in the query-row layout, one softmax update per 16 keys,
// ds_bpermute shuffles -- ran 6 MFMAs against ~100 VALU per 16 keys: L 577 50.6 -> 33.2 us,
// 100 x L 197 63.8 -> 48.8 us per launch, profiles/r03c/vit_attn_ab.txt):
//  * O is accumulated transposed, O^T = V^T P^T (16x16x32: A = V^T by two transposed LDS reads,
//    B = P^T straight from the S^T registers), so a lane holds its own query's O entries and the
//    softmax rescale needs no cross-lane broadcast; the row sum l stays lane-partial until the end;
//  * one softmax update per 32 keys (4 S MFMAs, 8 scores per lane), max over the 4 lane groups by
//    v_permlane32/16_swap (VALU, no LDS), scores in the log2 domain (exp2);
//  * the rescale of O is skipped when no query's running max moved (wave vote);
//  * the next 64-key K/V chunk is loaded into registers while the current one is consumed.
// Key slot 8 g4 + j of the PV MFMA is key 4 g4 + j (j < 4) or 16 + 4 g4 + j - 4 of the 32.
template <typename T>
__global__ __launch_bounds__(256) void attn_fwd_mfma_t(int nseq, int L, int H, int causal,
                                                       const T* __restrict__ qkv, int ldq,
                                                       T* __restrict__ out, int ldo,
                                                       float* __restrict__ lse) {
  __shared__ CLIPK_LDS_ALIGN short sK[64 * TRS];
  __shared__ CLIPK_LDS_ALIGN short sV[64 * TRS];
  constexpr float kLog2e = 1.4426950408889634f;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int h = blockIdx.y, s = blockIdx.z;
  const int W = H * 64;
  const size_t row0 = (size_t)s * L;
  const int q0 = blockIdx.x * 64 + w * 16;
  const int qr = q0 + r16;
  const bool qok = qr < L;
  const T* qp = qkv + (row0 + (qok ? qr : 0)) * ldq + h * 64;
  s16x8 qf[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) qf[kk] = ld_row16(qp + 8 * g4 + 32 * kk, qok);

  f32x4 o[4];  // o[t][r] = O[query r16][dim 16 t + 4 g4 + r]
#pragma unroll
  for (int t = 0; t < 4; ++t) o[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;  // running max (log2 domain, replicated over g4), lane-partial sum
  const int qmax = min(L, (int)(blockIdx.x + 1) * 64) - 1;
  const int kend = causal ? qmax + 1 : L;
  // K / V chunk staging: thread tid moves 16 B of rows (tid >> 3) and 32 + (tid >> 3)
  s16x8 rk[2], rv[2];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int rr = it * 32 + (tid >> 3), ch = tid & 7;
      const int kr = k0 + rr;
      const bool ok = kr < L;
      const T* base = qkv + (row0 + (ok ? kr : 0)) * ldq + h * 64 + ch * 8;
      rk[it] = ld_row16(base + W, ok);
      rv[it] = ld_row16(base + 2 * W, ok);
    }
  };
  fetch(0);
  const float sc2 = kScale * kLog2e;
  for (int k0 = 0; k0 < kend; k0 += 64) {
    __syncthreads();  // the previous chunk's readers are done
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int rr = it * 32 + (tid >> 3), ch = tid & 7;
      *reinterpret_cast<s16x8*>(sK + rr * TRS + ch * 8) = rk[it];
      *reinterpret_cast<s16x8*>(sV + rr * TRS + ch * 8) = rv[it];
    }
    __syncthreads();
    if (k0 + 64 < kend) fetch(k0 + 64);  // in flight while this chunk is consumed
    const int npair = min(2, (kend - k0 + 31) / 32);
    for (int pc = 0; pc < npair; ++pc) {
      const int kb = pc * 32;  // first key of the 32 within the chunk
      float sv[8];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        f32x4 st = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const s16x8 kf = *reinterpret_cast<const s16x8*>(sK + (kb + sub * 16 + r16) * TRS + 8 * g4 + 32 * kk);
          st = mfma32_t<T>(kf, qf[kk], st);  // st[r] = S[query r16][key kb + 16 sub + 4 g4 + r]
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) sv[4 * sub + r] = st[r] * sc2;
      }
      const int kabs = k0 + kb;
      if (kabs + 32 > L || (causal && kabs + 31 > q0)) {  // wave-uniform: edge chunk only
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int key = kabs + (j < 4 ? 4 * g4 + j : 16 + 4 * g4 + j - 4);
          if (key >= L || (causal && key > qr)) sv[j] = -INFINITY;
        }
      }
      float mx = sv[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) mx = fmaxf(mx, sv[j]);
      mx = xmax4(mx);
      const float mn = fmaxf(m, mx);
      const float msafe = mn == -INFINITY ? 0.f : mn;
      float p[8], ps = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        p[j] = __builtin_amdgcn_exp2f(sv[j] - msafe);
        ps += p[j];
      }
      if (__builtin_amdgcn_ballot_w64(mn > m) != 0) {  // some query's max moved: rescale
        const float corr = __builtin_amdgcn_exp2f(m - msafe);  // m = -inf -> 0 (O, l are 0)
        l *= corr;
#pragma unroll
        for (int t = 0; t < 4; ++t) o[t] *= corr;
      }
      l += ps;
      m = mn;
      typedef T t8 __attribute__((ext_vector_type(8)));
      t8 pv;
#pragma unroll
      for (int j = 0; j < 8; ++j) pv[j] = (T)p[j];
      const s16x8 pb = __builtin_bit_cast(s16x8, pv);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const s16x4 lo = tr_read(sV, kb + 4 * g4, 16 * t, lane), hi = tr_read(sV, kb + 16 + 4 * g4, 16 * t, lane);
        const s16x8 va = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        o[t] = mfma32_t<T>(va, pb, o[t]);
      }
    }
  }
  const float lt = xsum4(l);
  const float inv = 1.0f / lt;
  if (qok) {
    T* op = out + (row0 + qr) * ldo + h * 64 + 4 * g4;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      *reinterpret_cast<s16x4*>(op + 16 * t) = pack4<T>(o[t][0] * inv, o[t][1] * inv, o[t][2] * inv, o[t][3] * inv);
    if (lse && g4 == 0) lse[(row0 + qr) * H + h] = (m + __log2f(lt)) * 0.6931471805599453f;
  }
}

// ------------------------------------------------------------------ backward, any L (vision)
// The ViT's input-grad backward (deep visual prompts, IVLP / MaPLe / PromptSRC: model.py:
// 191-331, 401-431): L = 50..600 rows per sequence, non-causal (causal supported). Two passes
// that each recompute P from the saved log-sum-exp, so no atomics and no workspace:
//   pass KV -- a wave owns a 16-key tile j and sweeps the query tiles i: dK_j += dS^T Q_i,
//              dV_j += P^T dO_i (accumulators in registers, as the shared-prefix kernel's
//              prefix keys);
//   pass Q  -- a wave owns a 16-query tile i and sweeps the key tiles j: dQ_i += dS K_j.
// D_i = rowsum(dO_i o O_i) from the saved forward output (the row's keys span many tiles).
template <typename T, typename TG>
__device__ __forceinline__ float row_D(const TG* dor, const T* orow, bool ok, int g4) {
  // lane (r16, g4) holds 16 of row r16's 64 columns (8 g4 + 32 kk .. +7); reduce over g4
  float acc = 0.f;
  if (ok) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      float a[8], b[8];
      load16_f32<TG>(dor + 8 * g4 + 32 * kk, a);
      load16_f32<T>(orow + 8 * g4 + 32 * kk, b);
#pragma unroll
      for (int c = 0; c < 8; ++c) acc = fmaf(a[c], b[c], acc);
    }
  }
  acc += __shfl_xor(acc, 16, 64);
  acc += __shfl_xor(acc, 32, 64);
  return acc;
}

template <typename T, typename TG>
__global__ __launch_bounds__(256) void attn_bwd_long_kv(int nseq, int L, int H, int causal,
                                                        const T* __restrict__ qkv, int ldq,
                                                        const T* __restrict__ o_fwd, int ldof,
                                                        const TG* __restrict__ dout, int lddo,
                                                        const float* __restrict__ lse,
                                                        TG* __restrict__ dqkv, int lddq) {
  __shared__ CLIPK_LDS_ALIGN short sm[4][2][16 * TRS];  // per wave: Q_i, dO_i (transposed reads)
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int h = blockIdx.y, s = blockIdx.z, W = H * 64;
  const size_t row0 = (size_t)s * L;
  const int j0 = blockIdx.x * 64 + w * 16;
  if (j0 >= L) return;  // wave-uniform; no block barriers below
  short* tQ = sm[w][0];
  short* tD = sm[w][1];
  const int kr = min(j0 + r16, L - 1);
  const bool kok = j0 + r16 < L;
  s16x8 kp[2], vp[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const T* kb = qkv + (row0 + kr) * ldq + h * 64 + 8 * g4 + 32 * kk;
    kp[kk] = to_g8<T, TG>(*reinterpret_cast<const s16x8*>(kb + W));
    vp[kk] = to_g8<T, TG>(*reinterpret_cast<const s16x8*>(kb + 2 * W));
  }
  f32x4 dkp[4], dvp[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    dkp[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    dvp[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  const int nt = (L + 15) / 16;
  for (int it = causal ? j0 / 16 : 0; it < nt; ++it) {
    const int i0 = it * 16;
    const int qr = min(i0 + r16, L - 1);
    const T* qb = qkv + (row0 + qr) * ldq + h * 64;
    const TG* db = dout + (row0 + qr) * lddo + h * 64;
    s16x8 q[2], d[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      q[kk] = to_g8<T, TG>(*reinterpret_cast<const s16x8*>(qb + 8 * g4 + 32 * kk));
      d[kk] = *reinterpret_cast<const s16x8*>(db + 8 * g4 + 32 * kk);
    }
    const float Drow = row_D<T, TG>(db, o_fwd + (row0 + qr) * ldof + h * 64, true, g4);  // row r16
    float l1[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) l1[r] = lse[(row0 + min(i0 + 4 * g4 + r, L - 1)) * H + h];
    lds_fence_a();  // the previous tile's transposed reads are done
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      *reinterpret_cast<s16x8*>(tQ + r16 * TRS + 8 * g4 + 32 * kk) = q[kk];
      *reinterpret_cast<s16x8*>(tD + r16 * TRS + 8 * g4 + 32 * kk) = d[kk];
    }
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    f32x4 s1 = z, p1 = z;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      s1 = mfma32_t<TG>(q[kk], kp[kk], s1);  // S [i = 4g4+r][j = r16]
      p1 = mfma32_t<TG>(d[kk], vp[kk], p1);  // dP[i][j]
    }
    float P1[4], dS1[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * g4 + r;
      const bool ok = i < L && kok && !(causal && j0 + r16 > i);
      const float Di = __shfl(Drow, 4 * g4 + r, 64);
      P1[r] = ok ? __expf(s1[r] * kScale - l1[r]) : 0.f;
      dS1[r] = P1[r] * (p1[r] - Di);
    }
    const s16x4 bP = pack4<TG>(P1[0], P1[1], P1[2], P1[3]);
    const s16x4 bS = pack4<TG>(dS1[0], dS1[1], dS1[2], dS1[3]);
    lds_fence_a();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      dkp[t] = mfma16_t<TG>(tr_read(tQ, 4 * g4, 16 * t, lane), bS, dkp[t]);
      dvp[t] = mfma16_t<TG>(tr_read(tD, 4 * g4, 16 * t, lane), bP, dvp[t]);
    }
  }
  TG* orow = dqkv + (row0 + j0 + r16) * lddq + h * 64;
  store_tile64<TG>(orow + W, dkp, kScale, kok);
  store_tile64<TG>(orow + 2 * W, dvp, 1.0f, kok);
}

template <typename T, typename TG>
__global__ __launch_bounds__(256) void attn_bwd_long_q(int nseq, int L, int H, int causal,
                                                       const T* __restrict__ qkv, int ldq,
                                                       const T* __restrict__ o_fwd, int ldof,
                                                       const TG* __restrict__ dout, int lddo,
                                                       const float* __restrict__ lse,
                                                       TG* __restrict__ dqkv, int lddq) {
  __shared__ CLIPK_LDS_ALIGN short sm[4][16 * TRS];  // per wave: K_j (transposed reads)
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int h = blockIdx.y, s = blockIdx.z, W = H * 64;
  const size_t row0 = (size_t)s * L;
  const int i0 = blockIdx.x * 64 + w * 16;
  if (i0 >= L) return;  // wave-uniform
  short* tK = sm[w];
  const int qr = min(i0 + r16, L - 1);
  const bool qok = i0 + r16 < L;
  const T* qb = qkv + (row0 + qr) * ldq + h * 64;
  const TG* db = dout + (row0 + qr) * lddo + h * 64;
  s16x8 q[2], d[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    q[kk] = to_g8<T, TG>(*reinterpret_cast<const s16x8*>(qb + 8 * g4 + 32 * kk));
    d[kk] = *reinterpret_cast<const s16x8*>(db + 8 * g4 + 32 * kk);
  }
  const float D2 = row_D<T, TG>(db, o_fwd + (row0 + qr) * ldof + h * 64, true, g4);
  const float l2 = lse[(row0 + qr) * H + h];
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int jt_end = causal ? (min(i0 + 15, L - 1)) / 16 + 1 : (L + 15) / 16;
  for (int jt = 0; jt < jt_end; ++jt) {
    const int j0 = jt * 16;
    const int kr = min(j0 + r16, L - 1);
    const T* kb = qkv + (row0 + kr) * ldq + h * 64;
    s16x8 k[2], v[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      k[kk] = to_g8<T, TG>(*reinterpret_cast<const s16x8*>(kb + W + 8 * g4 + 32 * kk));
      v[kk] = to_g8<T, TG>(*reinterpret_cast<const s16x8*>(kb + 2 * W + 8 * g4 + 32 * kk));
    }
    lds_fence_a();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) *reinterpret_cast<s16x8*>(tK + r16 * TRS + 8 * g4 + 32 * kk) = k[kk];
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    f32x4 s2 = z, p2 = z;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      s2 = mfma32_t<TG>(k[kk], q[kk], s2);  // S^T[j = 4g4+r][i = r16]
      p2 = mfma32_t<TG>(v[kk], d[kk], p2);  // dP^T
    }
    float dS2[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = j0 + 4 * g4 + r;
      const bool ok = qok && j < L && !(causal && j > i0 + r16);
      const float P2 = ok ? __expf(s2[r] * kScale - l2) : 0.f;
      dS2[r] = P2 * (p2[r] - D2);
    }
    const s16x4 bT = pack4<TG>(dS2[0], dS2[1], dS2[2], dS2[3]);
    lds_fence_a();
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = mfma16_t<TG>(tr_read(tK, 4 * g4, 16 * t, lane), bT, acc[t]);
  }
  store_tile64<TG>(dqkv + (row0 + i0 + r16) * lddq + h * 64, acc, kScale, qok);
}

// VALU form (PREC fp32, and any dtype pair): 64 rows per block (lane = row), the other side
// streamed through LDS in chunks of 64 rows (row stride 65 floats where lanes read their own
// row: conflict-free column access).
template <typename T, typename TG>
__global__ __launch_bounds__(64) void attn_bwd_long_valu_q(int nseq, int L, int H, int causal,
                                                           const T* __restrict__ qkv, int ldq,
                                                           const T* __restrict__ o_fwd, int ldof,
                                                           const TG* __restrict__ dout, int lddo,
                                                           const float* __restrict__ lse,
                                                           TG* __restrict__ dqkv, int lddq) {
  __shared__ float sK[64 * 64], sV[64 * 64];
  const int lane = threadIdx.x, h = blockIdx.y, s = blockIdx.z, W = H * 64;
  const size_t row0 = (size_t)s * L;
  const int i = blockIdx.x * 64 + lane;
  const bool qok = i < L;
  const size_t row = row0 + (qok ? i : L - 1);
  float q[64], dO[64], acc[64];
  load_row64<T>(qkv + row * ldq + h * 64, q);
#pragma unroll
  for (int d = 0; d < 64; ++d) q[d] *= kScale;
  load_row64<TG>(dout + row * lddo + h * 64, dO);
  load_row64<T>(o_fwd + row * ldof + h * 64, acc);
  const float Di = dot64(dO, acc);
  const float li = lse[row * H + h];
#pragma unroll
  for (int d = 0; d < 64; ++d) acc[d] = 0.f;
  const int kend = causal ? min(L, (int)blockIdx.x * 64 + 64) : L;
  for (int k0 = 0; k0 < kend; k0 += 64) {
    __syncthreads();
    {
      const size_t kr = row0 + min(k0 + lane, L - 1);
#pragma unroll
      for (int c = 0; c < 64; c += 8) {
        float t[8];
        load_cols8<T>(qkv + kr * ldq + W + h * 64 + c, t);
#pragma unroll
        for (int d = 0; d < 8; ++d) sK[lane * 64 + c + d] = t[d];
        load_cols8<T>(qkv + kr * ldq + 2 * W + h * 64 + c, t);
#pragma unroll
        for (int d = 0; d < 8; ++d) sV[lane * 64 + c + d] = t[d];
      }
    }
    __syncthreads();
    const int nj = min(64, kend - k0);
    for (int jj = 0; jj < nj; ++jj) {
      const int j = k0 + jj;
      if (causal && j > i) continue;
      const float p = __expf(dot64(q, &sK[jj * 64]) - li);
      const float ds = p * (dot64(dO, &sV[jj * 64]) - Di);
#pragma unroll
      for (int d = 0; d < 64; ++d) acc[d] = fmaf(ds, sK[jj * 64 + d], acc[d]);
    }
  }
  if (qok) {
#pragma unroll
    for (int d = 0; d < 64; ++d) acc[d] *= kScale;
    store_row64<TG>(dqkv + row * lddq + h * 64, acc);
  }
}

template <typename T, typename TG>
__global__ __launch_bounds__(64) void attn_bwd_long_valu_kv(int nseq, int L, int H, int causal,
                                                            const T* __restrict__ qkv, int ldq,
                                                            const T* __restrict__ o_fwd, int ldof,
                                                            const TG* __restrict__ dout, int lddo,
                                                            const float* __restrict__ lse,
                                                            TG* __restrict__ dqkv, int lddq) {
  __shared__ float sQ[64 * 64], sO[64 * 64], sVo[64 * 65];
  __shared__ float sL[64], sD[64];
  const int lane = threadIdx.x, h = blockIdx.y, s = blockIdx.z, W = H * 64;
  const size_t row0 = (size_t)s * L;
  const int j = blockIdx.x * 64 + lane;
  const bool kok = j < L;
  const size_t krow = row0 + (kok ? j : L - 1);
  float k[64], dk[64], dv[64];
  load_row64<T>(qkv + krow * ldq + W + h * 64, k);
  load_row64<T>(qkv + krow * ldq + 2 * W + h * 64, dv);
#pragma unroll
  for (int d = 0; d < 64; ++d) {
    sVo[lane * 65 + d] = dv[d];
    dk[d] = 0.f;
    dv[d] = 0.f;
  }
  (void)sVo[0];
  const int q_begin = causal ? (int)blockIdx.x * 64 : 0;
  for (int q0 = q_begin; q0 < L; q0 += 64) {
    __syncthreads();
    {
      // staged in 8-column pieces (k, dk, dv stay live: keep the temporaries small)
      const size_t qr = row0 + min(q0 + lane, L - 1);
      float Dsum = 0.f;
#pragma unroll
      for (int c = 0; c < 64; c += 8) {
        float t[8], u[8];
        load_cols8<T>(qkv + qr * ldq + h * 64 + c, t);
#pragma unroll
        for (int d = 0; d < 8; ++d) sQ[lane * 64 + c + d] = t[d] * kScale;
        load_cols8<TG>(dout + qr * lddo + h * 64 + c, t);
        load_cols8<T>(o_fwd + qr * ldof + h * 64 + c, u);
#pragma unroll
        for (int d = 0; d < 8; ++d) {
          Dsum = fmaf(t[d], u[d], Dsum);
          sO[lane * 64 + c + d] = t[d];  // dO rows
        }
      }
      sD[lane] = Dsum;
      sL[lane] = lse[qr * H + h];
    }
    __syncthreads();
    const int ni = min(64, L - q0);
    for (int ii = 0; ii < ni; ++ii) {
      const int i = q0 + ii;
      if (causal && j > i) continue;
      const float* qr = &sQ[ii * 64];
      const float* dor = &sO[ii * 64];
      const float p = __expf(dot64(qr, k) - sL[ii]);
      float dp = 0.f;
#pragma unroll
      for (int d = 0; d < 64; ++d) dp = fmaf(dor[d], sVo[lane * 65 + d], dp);
      const float ds = p * (dp - sD[ii]);
#pragma unroll
      for (int d = 0; d < 64; ++d) {
        dv[d] = fmaf(p, dor[d], dv[d]);
        dk[d] = fmaf(ds, qr[d], dk[d]);
      }
    }
  }
  if (kok) {
    store_row64<TG>(dqkv + krow * lddq + W + h * 64, dk);
    store_row64<TG>(dqkv + krow * lddq + 2 * W + h * 64, dv);
  }
}

template <typename T>
static int launch_fwd(int nseq, int L, int H, int causal, const void* qkv, int ldq, void* out,
                      int ldo, float* lse, hipStream_t st) {
  const int pairs = nseq * H;
  auto short_launch = [&](auto lp_tag) {
    constexpr int LP = decltype(lp_tag)::value;
    constexpr int G = 64 / LP;
    const int blocks = (pairs + 4 * G - 1) / (4 * G);
    hipLaunchKernelGGL((attn_fwd_short<LP, T>), dim3(blocks), dim3(256), 0, st, nseq, L, H, causal,
                       (const T*)qkv, ldq, (T*)out, ldo, lse);
  };
  if constexpr (sizeof(T) == 2) {
    if (L > 16) {  // MFMA flash forward (vision L = 50..577, text 16 < L <= 77)
      dim3 grid((L + 63) / 64, H, nseq);
      hipLaunchKernelGGL((attn_fwd_mfma_t<T>), grid, dim3(256), 0, st, nseq, L, H, causal, (const T*)qkv, ldq,
                         (T*)out, ldo, lse);
      CLIPK_CHECK_LAUNCH();
      return CLIPK_OK;
    }
  }
  if (L <= 16) short_launch(std::integral_constant<int, 16>{});
  else if (L <= 32) short_launch(std::integral_constant<int, 32>{});
  else if (L <= 64) short_launch(std::integral_constant<int, 64>{});
  else {
    static_assert(sizeof(T) == 2 || __is_same(T, float), "fp32 long forward");
    if constexpr (__is_same(T, float)) {
      dim3 grid((L + 63) / 64, H, nseq);
      hipLaunchKernelGGL(attn_fwd_f32, grid, dim3(256), 0, st, nseq, L, H, causal, (const float*)qkv, ldq,
                         (float*)out, ldo, lse);
    }
  }
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

// 16 < L <= 64 with 16-bit operands (CoOp n_ctx 16: L_eff 23): the two-pass MFMA kernels
// instead of the VALU attn_bwd_short (knob CLIPK_ATTN_MFMA_BWD, default on)
static bool mfma_long_bwd() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLIPK_ATTN_MFMA_BWD");
    v = e ? atoi(e) : 1;
  }
  return v != 0;
}

template <typename T, typename TG>
static int launch_bwd(int nseq, int L, int H, int causal, const void* qkv, int ldq,
                      const void* ofwd, int ldof, const void* dout, int lddo, const float* lse,
                      void* dqkv, int lddq, hipStream_t st) {
  const int pairs = nseq * H;
  if constexpr (sizeof(TG) == 2 && sizeof(T) == 2) {
    if (L <= 16) {
      hipLaunchKernelGGL((attn_bwd_mfma16<T, TG>), dim3((pairs + 3) / 4), dim3(256), 0, st, nseq, L, H,
                         causal, (const T*)qkv, ldq, (const TG*)dout, lddo, lse, (TG*)dqkv, lddq);
      CLIPK_CHECK_LAUNCH();
      return CLIPK_OK;
    }
  }
  if (L > 64 || (sizeof(TG) == 2 && sizeof(T) == 2 && mfma_long_bwd())) {
    // two passes (dK/dV per key tile, dQ per query tile); MFMA for 16-bit operands
    if constexpr (sizeof(TG) == 2 && sizeof(T) == 2) {
      dim3 grid((L + 63) / 64, H, nseq);
      hipLaunchKernelGGL((attn_bwd_long_kv<T, TG>), grid, dim3(256), 0, st, nseq, L, H, causal, (const T*)qkv, ldq,
                         (const T*)ofwd, ldof, (const TG*)dout, lddo, lse, (TG*)dqkv, lddq);
      CLIPK_CHECK_LAUNCH();
      hipLaunchKernelGGL((attn_bwd_long_q<T, TG>), grid, dim3(256), 0, st, nseq, L, H, causal, (const T*)qkv, ldq,
                         (const T*)ofwd, ldof, (const TG*)dout, lddo, lse, (TG*)dqkv, lddq);
    } else {
      dim3 grid((L + 63) / 64, H, nseq);
      hipLaunchKernelGGL((attn_bwd_long_valu_kv<T, TG>), grid, dim3(64), 0, st, nseq, L, H, causal,
                         (const T*)qkv, ldq, (const T*)ofwd, ldof, (const TG*)dout, lddo, lse, (TG*)dqkv, lddq);
      CLIPK_CHECK_LAUNCH();
      hipLaunchKernelGGL((attn_bwd_long_valu_q<T, TG>), grid, dim3(64), 0, st, nseq, L, H, causal,
                         (const T*)qkv, ldq, (const T*)ofwd, ldof, (const TG*)dout, lddo, lse, (TG*)dqkv, lddq);
    }
    CLIPK_CHECK_LAUNCH();
    return CLIPK_OK;
  }
  auto go = [&](auto lp_tag) {
    constexpr int LP = decltype(lp_tag)::value;
    constexpr int G = 64 / LP;
    const int blocks = (pairs + G - 1) / G;
    hipLaunchKernelGGL((attn_bwd_short<LP, T, TG>), dim3(blocks), dim3(64), 0, st, nseq, L, H,
                       causal, (const T*)qkv, ldq, (const T*)ofwd, ldof, (const TG*)dout, lddo, lse,
                       (TG*)dqkv, lddq);
  };
  if (L <= 16) go(std::integral_constant<int, 16>{});
  else if (L <= 32) go(std::integral_constant<int, 32>{});
  else if (L <= 64) go(std::integral_constant<int, 64>{});
  else return CLIPK_ESHAPE;
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

}  // namespace clipk

using namespace clipk;

extern "C" int clipk_attention_fwd(int dtype, int nseq, int L, int heads, int causal,
                                   const void* qkv, int ldqkv, void* out, int ldo, float* lse,
                                   void* stream) {
  if (!qkv || !out) return CLIPK_EINVAL;
  if (nseq < 0 || L <= 0 || heads <= 0 || ldqkv < 3 * heads * 64 || ldo < heads * 64 || ldqkv % 8 ||
      ldo % 8)
    return CLIPK_ESHAPE;
  if (nseq == 0) return CLIPK_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case CLIPK_F16: return launch_fwd<f16>(nseq, L, heads, causal, qkv, ldqkv, out, ldo, lse, st);
    case CLIPK_BF16: return launch_fwd<bf16>(nseq, L, heads, causal, qkv, ldqkv, out, ldo, lse, st);
    case CLIPK_F32: return launch_fwd<float>(nseq, L, heads, causal, qkv, ldqkv, out, ldo, lse, st);
    default: return CLIPK_EDTYPE;
  }
}

extern "C" int clipk_attention_bwd(int dtype, int grad_dtype, int nseq, int L, int heads,
                                    int causal, const void* qkv, int ldqkv, const void* ofwd,
                                    int ldof, const void* dout, int lddo, const float* lse,
                                    void* dqkv, int lddqkv, void* stream) {
  if (!qkv || !ofwd || !dout || !lse || !dqkv) return CLIPK_EINVAL;
  if (nseq < 0 || L <= 0 || heads <= 0 || ldqkv < 3 * heads * 64 || lddqkv < 3 * heads * 64 ||
      ldof < heads * 64 || lddo < heads * 64)
    return CLIPK_ESHAPE;
  if (nseq == 0) return CLIPK_OK;
  hipStream_t st = (hipStream_t)stream;
#define CLIPK_BWD(TT, TGG) \
  return launch_bwd<TT, TGG>(nseq, L, heads, causal, qkv, ldqkv, ofwd, ldof, dout, lddo, lse, dqkv, lddqkv, st)
  if (dtype == CLIPK_F16 && grad_dtype == CLIPK_BF16) CLIPK_BWD(f16, bf16);
  if (dtype == CLIPK_F16 && grad_dtype == CLIPK_F16) CLIPK_BWD(f16, f16);
  if (dtype == CLIPK_BF16 && grad_dtype == CLIPK_BF16) CLIPK_BWD(bf16, bf16);
  if (dtype == CLIPK_F32 && grad_dtype == CLIPK_F32) CLIPK_BWD(float, float);
#undef CLIPK_BWD
  return CLIPK_EDTYPE;
}
