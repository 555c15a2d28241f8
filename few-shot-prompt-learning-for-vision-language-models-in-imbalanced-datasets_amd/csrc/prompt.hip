// Small HBM-bound kernels on the CoOp/CoCoOp path: patch extraction, ViT embedding +
// ln_pre, prompt assembly (+pos) and its ctx gradient, cosine logits fwd/bwd, CE/focal
// loss fwd+bwd, CoCoOp Meta-Net fwd/bwd, fused SGD, casts. One wave per row throughout,
// float4 accesses, fixed-order (deterministic) reductions.
#include <type_traits>

#include "common.h"

namespace clipk {

// ---------------------------------------------------------------- im2col (conv1 as GEMM)
// model.py:376,402: Conv2d(3, D, kernel=p, stride=p, bias=False)
template <typename TO>
__global__ __launch_bounds__(256) void im2col_kernel(int B, int R, int P, int Kp,
                                                     const float* __restrict__ img,
                                                     TO* __restrict__ out) {
  const int G = R / P;
  const long total = (long)B * G * G * Kp;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int k = (int)(e % Kp);
    const long patch = e / Kp;
    float v = 0.f;
    if (k < 3 * P * P) {
      const int b = (int)(patch / (G * G)), pi = (int)(patch % (G * G));
      const int gy = pi / G, gx = pi % G;
      const int c = k / (P * P), r = k % (P * P), ky = r / P, kx = r % P;
      v = img[(((long)b * 3 + c) * R + gy * P + ky) * R + gx * P + kx];
    }
    out[e] = (TO)v;
  }
}

// ---------------------------------------------------------------- ViT embed + ln_pre
// model.py:405-420: x = cat(cls, patches) + pos; ln_pre(x). One wave per token row.
// n_vpt > 0 (IVLP / MaPLe / PromptSRC, model.py:413-420 / 465-472): n_vpt visual prompt rows
// appended after the L image tokens (no positional embedding), rows per image L + n_vpt.
__global__ __launch_bounds__(256) void vit_embed_ln_kernel(int B, int L, int n_vpt, int D,
                                                           const float* __restrict__ patch,
                                                           const float* __restrict__ cls,
                                                           const float* __restrict__ pos,
                                                           const float* __restrict__ vpt,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           float* __restrict__ x) {
  const int lane = threadIdx.x & 63;
  const int Lo = L + n_vpt;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B * Lo) return;
  const int b = r / Lo, t = r % Lo;
  const bool prompt = t >= L;
  const float* src = prompt ? vpt + (size_t)(t - L) * D : t == 0 ? cls : patch + ((size_t)b * (L - 1) + t - 1) * D;
  const float* pp = pos + (size_t)(prompt ? 0 : t) * D;
  const int nv = D >> 2;
  f32x4 v[4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + i * 64;
    if (c < nv) {
      v[i] = reinterpret_cast<const f32x4*>(src)[c];
      if (!prompt) v[i] += reinterpret_cast<const f32x4*>(pp)[c];
      s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
    }
  }
  const float mu = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + i * 64;
    if (c < nv)
#pragma unroll
      for (int k = 0; k < 4; ++k) { const float d = v[i][k] - mu; q += d * d; }
  }
  const float rs = rsqrtf(wave_sum(q) / D + 1e-5f);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + i * 64;
    if (c < nv) {
      const f32x4 gg = reinterpret_cast<const f32x4*>(gamma)[c];
      const f32x4 bb = reinterpret_cast<const f32x4*>(beta)[c];
      f32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = (v[i][k] - mu) * rs * gg[k] + bb[k];
      reinterpret_cast<f32x4*>(x + (size_t)r * D)[c] = o;
    }
  }
}

// ---------------------------------------------------------------- prompt assembly
// PromptLearner.forward (coop.py:259-296 / cocoop.py:173-198) + TextEncoder pos add
// (coop.py:197), truncated to L tokens. src_map[c*L+t] >= 0: fixed token-embedding row
// (prefix / class-name / suffix), < 0: context slot (-1-m).
__global__ __launch_bounds__(256) void prompt_assemble_kernel(int B, int C, int L, int W,
                                                              const int* __restrict__ src_map,
                                                              const float* __restrict__ emb,
                                                              const float* __restrict__ ctx, long sb,
                                                              long sc, const float* __restrict__ bias,
                                                              const float* __restrict__ pos,
                                                              float* __restrict__ x0) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= (long)B * C * L) return;
  const int t = (int)(r % L);
  const long s = r / L;
  const int c = (int)(s % C), b = (int)(s / C);
  const int m = src_map[c * L + t];
  const float* src = m >= 0 ? emb + ((size_t)c * 77 + m) * W : ctx + b * sb + c * sc + (size_t)(-1 - m) * W;
  const bool add_bias = m < 0 && bias != nullptr;
  const float* bp = bias + (size_t)b * W;
  const float* pp = pos + (size_t)t * W;
  float* dst = x0 + r * W;
  for (int c4 = lane; c4 < W / 4; c4 += 64) {
    f32x4 v = reinterpret_cast<const f32x4*>(src)[c4] + reinterpret_cast<const f32x4*>(pp)[c4];
    if (add_bias) v += reinterpret_cast<const f32x4*>(bp)[c4];
    reinterpret_cast<f32x4*>(dst)[c4] = v;
  }
}

// d ctx: out[(b*(csc?C:1) + cc)*n_ctx + k][w] = sum_{c in group} dx0[((b*C+c)*L + ctx_pos[c*n_ctx+k])*W + w]
// Block = (output row, 64 columns); wave v sums classes c = v, v+4, ... in order, then the 4
// partials are added in a fixed order (deterministic).
__global__ __launch_bounds__(256) void ctx_grad_kernel(int B, int C, int L, int W, int n_ctx, int csc,
                                                       const int* __restrict__ ctx_pos,
                                                       const float* __restrict__ dx0,
                                                       float* __restrict__ dctx) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wcol = blockIdx.y * 64 + lane;
  const int o = blockIdx.x;  // output row
  const int k = o % n_ctx;
  const int grp = o / n_ctx;
  int b, c0, c1;
  if (csc) { b = grp / C; c0 = grp % C; c1 = c0 + 1; } else { b = grp; c0 = 0; c1 = C; }
  float acc = 0.f;
  if (wcol < W) {
#pragma unroll 4
    for (int c = c0 + wv; c < c1; c += 4) {
      const int t = ctx_pos[c * n_ctx + k];
      acc += dx0[(((size_t)b * C + c) * L + t) * W + wcol];
    }
  }
  red[wv][lane] = acc;
  __syncthreads();
  if (wv == 0 && wcol < W) dctx[(size_t)o * W + wcol] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// Shared-prefix packed prompts (see attention_prefix.hip): group g's row r holds token
// (c, t) = (row_tab[r] / L, row_tab[r] % L); same splice as prompt_assemble_kernel.
__global__ __launch_bounds__(256) void prompt_assemble_rows_kernel(int G, int R, int L, int W,
                                                                   const int* __restrict__ row_tab,
                                                                   const int* __restrict__ src_map,
                                                                   const float* __restrict__ emb,
                                                                   const float* __restrict__ ctx, long sb,
                                                                   long sc, const float* __restrict__ bias,
                                                                   const float* __restrict__ pos,
                                                                   float* __restrict__ x0) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= (long)G * R) return;
  const int g = (int)(r / R);
  const int ct = row_tab[r % R];
  const int c = ct / L, t = ct % L;
  const int m = src_map[ct];
  const float* src = m >= 0 ? emb + ((size_t)c * 77 + m) * W : ctx + g * sb + c * sc + (size_t)(-1 - m) * W;
  const bool add_bias = m < 0 && bias != nullptr;
  const float* bp = bias + (size_t)g * W;
  const float* pp = pos + (size_t)t * W;
  float* dst = x0 + r * W;
  for (int c4 = lane; c4 < W / 4; c4 += 64) {
    f32x4 v = reinterpret_cast<const f32x4*>(src)[c4] + reinterpret_cast<const f32x4*>(pp)[c4];
    if (add_bias) v += reinterpret_cast<const f32x4*>(bp)[c4];
    reinterpret_cast<f32x4*>(dst)[c4] = v;
  }
}

// d ctx on packed prompts: out[g*n_ctx + k] = sum of dx0 over the group rows listed for
// slot k (slot_rows[slot_ptr[k] .. slot_ptr[k+1]); a shared prefix row is listed once,
// since its gradient already sums every class). Fixed-order 4-wave reduction.
__global__ __launch_bounds__(256) void ctx_grad_rows_kernel(int R, int W, int n_ctx,
                                                            const int* __restrict__ slot_ptr,
                                                            const int* __restrict__ slot_rows,
                                                            const float* __restrict__ dx0,
                                                            float* __restrict__ dctx) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wcol = blockIdx.y * 64 + lane;
  const int o = blockIdx.x;
  const int k = o % n_ctx, g = o / n_ctx;
  float acc = 0.f;
  if (wcol < W) {
    const int e = slot_ptr[k + 1];
#pragma unroll 4
    for (int i = slot_ptr[k] + wv; i < e; i += 4) acc += dx0[((size_t)g * R + slot_rows[i]) * W + wcol];
  }
  red[wv][lane] = acc;
  __syncthreads();
  if (wv == 0 && wcol < W) dctx[(size_t)o * W + wcol] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// CoCoOp's ctx_shifted = ctx + bias_g on packed prompts (PromptAssembleFn.backward): the two sums
// of the per-(g, k) slot gradients in one launch, one thread per column w:
//   dctx[k, w] = sum_g d(g, k)[w]   (the shared ctx, summed over the images in g order)
//   dbias[g, w] = sum_k d(g, k)[w]  (the Meta-Net output of image g, summed over the slots)
// with d(g, k) = the ctx_grad_rows_kernel sum of slot k's rows of group g
__global__ __launch_bounds__(256) void ctx_bias_grad_rows_kernel(int G, int R, int W, int n_ctx,
                                                                 const int* __restrict__ slot_ptr,
                                                                 const int* __restrict__ slot_rows,
                                                                 const float* __restrict__ dx0,
                                                                 float* __restrict__ dctx,
                                                                 float* __restrict__ dbias) {
  const int w = blockIdx.x * 256 + threadIdx.x;
  if (w >= W) return;
  for (int k = 0; k < n_ctx; ++k) {
    const int i0 = slot_ptr[k], i1 = slot_ptr[k + 1];
    float sk = 0.f;
    for (int g = 0; g < G; ++g) {
      float d = 0.f;
      for (int i = i0; i < i1; ++i) d += dx0[((size_t)g * R + slot_rows[i]) * W + w];
      sk += d;
      if (dbias) dbias[(size_t)g * W + w] = (k == 0 ? 0.f : dbias[(size_t)g * W + w]) + d;
    }
    dctx[(size_t)k * W + w] = sk;
  }
}

// ---------------------------------------------------------------- cosine logits
// coop.py:356-363 / cocoop.py:238-251: logits = exp(logit_scale) * (imf/|imf|) . (txt/|txt|)
__global__ __launch_bounds__(256) void cos_logits_fwd_kernel(int B, int C, int E, int per_image,
                                                             float scale, const float* __restrict__ imf,
                                                             const float* __restrict__ txt,
                                                             float* __restrict__ logits,
                                                             float* __restrict__ inv_t,
                                                             float* __restrict__ inv_i) {
  const int lane = threadIdx.x & 63;
  const long pidx = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pidx >= (long)B * C) return;
  const int b = (int)(pidx / C), c = (int)(pidx % C);
  const long row = per_image ? pidx : c;
  const float* ip = imf + (size_t)b * E;
  const float* tp = txt + (size_t)row * E;
  float d = 0.f, ti = 0.f, ii = 0.f;
  for (int e = lane; e < E / 4; e += 64) {
    const f32x4 a = reinterpret_cast<const f32x4*>(ip)[e];
    const f32x4 t = reinterpret_cast<const f32x4*>(tp)[e];
#pragma unroll
    for (int k = 0; k < 4; ++k) { d += a[k] * t[k]; ti += t[k] * t[k]; ii += a[k] * a[k]; }
  }
  d = wave_sum(d); ti = wave_sum(ti); ii = wave_sum(ii);
  const float it = rsqrtf(ti), iv = rsqrtf(ii);
  if (lane == 0) {
    logits[pidx] = scale * d * it * iv;
    if (inv_t && (per_image || b == 0)) inv_t[row] = it;
    if (inv_i && c == 0) inv_i[b] = iv;
  }
}

// dtxt[row] = inv_t * (dy - y (y.dy)),  y = txt*inv_t,  dy = scale * sum_b dl[b,c] * imf_b*inv_i[b]
__global__ __launch_bounds__(256) void cos_logits_bwd_kernel(int B, int C, int E, int per_image,
                                                             float scale, const float* __restrict__ imf,
                                                             const float* __restrict__ txt,
                                                             const float* __restrict__ inv_t,
                                                             const float* __restrict__ inv_i,
                                                             const float* __restrict__ dl,
                                                             float* __restrict__ dtxt) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long nrows = per_image ? (long)B * C : C;
  if (row >= nrows) return;
  const int c = (int)(row % C);
  const int b0 = per_image ? (int)(row / C) : 0, b1 = per_image ? b0 + 1 : B;
  const float it = inv_t[row];
  const float* tp = txt + (size_t)row * E;
  constexpr int MAXE = 16;  // E <= 1024
  float dy[MAXE], y[MAXE];
  float yd = 0.f;
#pragma unroll
  for (int q = 0; q < MAXE; ++q) { dy[q] = 0.f; y[q] = 0.f; }
  for (int b = b0; b < b1; ++b) {
    const float coef = scale * dl[(size_t)b * C + c] * inv_i[b];
    const float* ip = imf + (size_t)b * E;
#pragma unroll
    for (int q = 0; q < MAXE; ++q) {
      const int e = lane + q * 64;
      if (e < E) dy[q] += coef * ip[e];
    }
  }
#pragma unroll
  for (int q = 0; q < MAXE; ++q) {
    const int e = lane + q * 64;
    if (e < E) { y[q] = tp[e] * it; yd += y[q] * dy[q]; }
  }
  yd = wave_sum(yd);
  float* op = dtxt + (size_t)row * E;
#pragma unroll
  for (int q = 0; q < MAXE; ++q) {
    const int e = lane + q * 64;
    if (e < E) op[e] = it * (dy[q] - y[q] * yd);
  }
}

// ---------------------------------------------------------------- CE / focal loss
// nn.CrossEntropyLoss (mean) and MultiClassFocalLoss (coop.py:145-163): FL = a_y (1-p)^g ce.
__global__ __launch_bounds__(64) void ce_loss_kernel(int B, int C, const float* __restrict__ logits,
                                                     const int64_t* __restrict__ labels,
                                                     const float* __restrict__ alpha, float gamma,
                                                     int focal, float grad_scale,
                                                     float* __restrict__ row_loss,
                                                     float* __restrict__ dlogits) {
  const int lane = threadIdx.x;
  const int b = blockIdx.x;
  const float* z = logits + (size_t)b * C;
  const int y = (int)labels[b];
  float mx = -INFINITY;
  for (int c = lane; c < C; c += 64) mx = fmaxf(mx, z[c]);
  mx = wave_max(mx);
  float se = 0.f;
  for (int c = lane; c < C; c += 64) se += __expf(z[c] - mx);
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  const float ce = lse - z[y];
  float wgt = 1.f, loss = ce;
  if (focal) {
    const float p = __expf(-ce);
    const float a = alpha ? alpha[y] : 1.f;
    const float om = 1.f - p;
    loss = a * powf(om, gamma) * ce;
    wgt = a * (powf(om, gamma) + (gamma != 0.f ? gamma * p * powf(om, gamma - 1.f) * ce : 0.f));
  }
  if (lane == 0 && row_loss) row_loss[b] = loss;
  if (dlogits) {
    for (int c = lane; c < C; c += 64) {
      const float pc = __expf(z[c] - lse);
      dlogits[(size_t)b * C + c] = grad_scale * wgt * (pc - (c == y ? 1.f : 0.f));
    }
  }
}

// The loss reduced in the same launch (clipk_ce_loss_reduce): one block, wave w takes rows w,
// w + 4, ...; the row losses are summed in row order by one thread (deterministic)
__global__ __launch_bounds__(256) void ce_loss_reduce_kernel(int B, int C, const float* __restrict__ logits,
                                                             const int64_t* __restrict__ labels,
                                                             const float* __restrict__ alpha, float gamma,
                                                             int focal, float grad_scale, int mean,
                                                             float* __restrict__ row_loss,
                                                             float* __restrict__ loss,
                                                             float* __restrict__ dlogits) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int b = wv; b < B; b += 4) {
    const float* z = logits + (size_t)b * C;
    const int y = (int)labels[b];
    float mx = -INFINITY;
    for (int c = lane; c < C; c += 64) mx = fmaxf(mx, z[c]);
    mx = wave_max(mx);
    float se = 0.f;
    for (int c = lane; c < C; c += 64) se += __expf(z[c] - mx);
    se = wave_sum(se);
    const float lse = mx + __logf(se);
    const float ce = lse - z[y];
    float wgt = 1.f, l = ce;
    if (focal) {
      const float p = __expf(-ce);
      const float a = alpha ? alpha[y] : 1.f;
      const float om = 1.f - p;
      l = a * powf(om, gamma) * ce;
      wgt = a * (powf(om, gamma) + (gamma != 0.f ? gamma * p * powf(om, gamma - 1.f) * ce : 0.f));
    }
    if (lane == 0) row_loss[b] = l;
    if (dlogits)
      for (int c = lane; c < C; c += 64) {
        const float pc = __expf(z[c] - lse);
        dlogits[(size_t)b * C + c] = grad_scale * wgt * (pc - (c == y ? 1.f : 0.f));
      }
  }
  __threadfence_block();
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += row_loss[b];
    loss[0] = mean ? s * (1.0f / (float)B) : s;  // (torch's mean: the sum times 1 / B)
  }
}

// ---------------------------------------------------------------- Meta-Net (cocoop.py:139-143)
// Block (image b, 64-output block ob): every block of an image recomputes the Hd hidden units
// (W1 stays in L2). Lane l of a wave holds x[b, 4 l .. 4 l + 3 (+ 256 i)] and the matching W1
// columns of up to 16 hidden units, all loaded before the first sum, so the wave pays one load
// round trip instead of one per hidden unit (the first form, a dependent load + wave sum per
// unit, took 23-24 us at any batch: a latency chain on the step's critical path). Then 4 lanes
// per output split the Hd-long second dot product (fixed order: 4 interleaved partial sums, then
// the quad sum). V % 256 == 0, V <= 1024, Hd <= 64, 16-B aligned x / W1 (the CLIP widths);
// other shapes run meta_net_fwd_generic_kernel.
// NORM (clipk_meta_net_fwd_norm): x is the raw image feature; every wave holds the whole row, so
// each forms |x| itself and the Meta-Net runs on x / |x| (cocoop.py:238's imf / imf.norm(), the
// row also written to xn by one wave for the cosine logits and the backward)
template <bool NORM>
__global__ __launch_bounds__(256) void meta_net_fwd_kernel(int V, int Hd, int Wd, const float* __restrict__ x,
                                                           const float* __restrict__ w1,
                                                           const float* __restrict__ b1,
                                                           const float* __restrict__ w2,
                                                           const float* __restrict__ b2,
                                                           float* __restrict__ xn,
                                                           float* __restrict__ h, float* __restrict__ y) {
  extern __shared__ float sh[];  // Hd floats
  const int b = blockIdx.x, ob = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nc = V / 256;  // float4 chunks per lane (1..4)
  const float* xb = x + (size_t)b * V;
  f32x4 xv[4], wk[16][4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (c < nc) xv[c] = *reinterpret_cast<const f32x4*>(xb + 4 * lane + 256 * c);
  if constexpr (NORM) {
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < nc)
#pragma unroll
        for (int e = 0; e < 4; ++e) ss = fmaf(xv[c][e], xv[c][e], ss);
    const float nrm = sqrtf(wave_sum(ss));
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < nc) {
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[c][e] = xv[c][e] / nrm;
        if (ob == 0 && wv == 0) *reinterpret_cast<f32x4*>(xn + (size_t)b * V + 4 * lane + 256 * c) = xv[c];
      }
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int k = wv + 4 * j;
    if (k < Hd) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < nc) wk[j][c] = *reinterpret_cast<const f32x4*>(w1 + (size_t)k * V + 4 * lane + 256 * c);
    }
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int k = wv + 4 * j;
    if (k < Hd) {
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < nc)
#pragma unroll
          for (int e = 0; e < 4; ++e) a = fmaf(wk[j][c][e], xv[c][e], a);
      a = fmaxf(wave_sum(a) + b1[k], 0.f);
      if (lane == 0) { sh[k] = a; if (h && ob == 0) h[(size_t)b * Hd + k] = a; }
    }
  }
  __syncthreads();
  const int o = ob * 64 + (tid >> 2), part = tid & 3;
  const bool ok = o < Wd;
  float a = 0.f;
  if (ok) {
#pragma unroll 16
    for (int k = part; k < Hd; k += 4) a += w2[(size_t)o * Hd + k] * sh[k];
  }
  a += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a), 0xB1, 0xF, 0xF, false));
  a += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a), 0x4E, 0xF, 0xF, false));
  if (ok && part == 0) y[(size_t)b * Wd + o] = a + b2[o];
}

// any V / Hd (tiny test models): one block per image, a dependent load + wave sum per hidden unit
// (NORM: x / |x| written to xn first, then read back: the block's own rows)
template <bool NORM>
__global__ __launch_bounds__(256) void meta_net_fwd_generic_kernel(int V, int Hd, int Wd, const float* __restrict__ x,
                                                                   const float* __restrict__ w1,
                                                                   const float* __restrict__ b1,
                                                                   const float* __restrict__ w2,
                                                                   const float* __restrict__ b2,
                                                                   float* __restrict__ xn,
                                                                   float* __restrict__ h, float* __restrict__ y) {
  extern __shared__ float sh[];  // Hd floats
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* xb = x + (size_t)b * V;
  if constexpr (NORM) {
    float ss = 0.f;
    for (int v = lane; v < V; v += 64) ss = fmaf(xb[v], xb[v], ss);
    const float nrm = sqrtf(wave_sum(ss));
    if (wv == 0)
      for (int v = lane; v < V; v += 64) xn[(size_t)b * V + v] = xb[v] / nrm;
    __threadfence_block();
    __syncthreads();
    xb = xn + (size_t)b * V;
  }
  for (int k = wv; k < Hd; k += 4) {
    float a = 0.f;
    for (int v = lane; v < V; v += 64) a += w1[(size_t)k * V + v] * xb[v];
    a = wave_sum(a) + b1[k];
    a = fmaxf(a, 0.f);
    if (lane == 0) { sh[k] = a; if (h) h[(size_t)b * Hd + k] = a; }
  }
  __syncthreads();
  for (int o = tid; o < Wd; o += 256) {
    float a = b2[o];
    for (int k = 0; k < Hd; ++k) a += w2[(size_t)o * Hd + k] * sh[k];
    y[(size_t)b * Wd + o] = a;
  }
}

// Meta-Net backward in two launches (every output element owned by one thread; fixed-order
// sums over the batch, deterministic):
//   A: waves [0, B*Hd): dh[b,k] = (dy[b] . W2[:,k]) * (h[b,k] > 0);
//      threads after that: dW2[o,k] = sum_b dy[b,o] h[b,k], db2[o] = sum_b dy[b,o]
//   B: dW1[k,v] = sum_b dh[b,k] x[b,v], db1[k] = sum_b dh[b,k]
__global__ __launch_bounds__(256) void meta_net_bwd_a_kernel(int B, int Hd, int Wd, int nb_dh,
                                                             const float* __restrict__ h,
                                                             const float* __restrict__ w2,
                                                             const float* __restrict__ dy,
                                                             float* __restrict__ dw2, float* __restrict__ db2,
                                                             float* __restrict__ dh) {
  const int tid = threadIdx.x, lane = tid & 63;
  if ((int)blockIdx.x < nb_dh) {
    const int bk = blockIdx.x * 4 + (tid >> 6);
    if (bk >= B * Hd) return;
    const int b = bk / Hd, k = bk % Hd;
    float a = 0.f;
    for (int o = lane; o < Wd; o += 64) a += dy[(size_t)b * Wd + o] * w2[(size_t)o * Hd + k];
    a = wave_sum(a);
    if (lane == 0) dh[bk] = h[bk] > 0.f ? a : 0.f;
    return;
  }
  const long i = (long)(blockIdx.x - nb_dh) * 256 + tid;
  if (i >= (long)Wd * Hd) return;
  const int o = (int)(i / Hd), k = (int)(i % Hd);
  float a = 0.f, s = 0.f;
  for (int b = 0; b < B; ++b) {
    const float d = dy[(size_t)b * Wd + o];
    a += d * h[(size_t)b * Hd + k];
    s += d;
  }
  dw2[i] = a;
  if (k == 0) db2[o] = s;
}

__global__ __launch_bounds__(256) void meta_net_bwd_b_kernel(int B, int V, int Hd,
                                                             const float* __restrict__ x,
                                                             const float* __restrict__ dh,
                                                             float* __restrict__ dw1, float* __restrict__ db1) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)Hd * V) return;
  const int k = (int)(i / V), v = (int)(i % V);
  float a = 0.f, s = 0.f;
  for (int b = 0; b < B; ++b) {
    const float d = dh[(size_t)b * Hd + k];
    a += d * x[(size_t)b * V + v];
    s += d;
  }
  dw1[i] = a;
  if (v == 0) db1[k] = s;
}

// ---------------------------------------------------------------- SGD (optimizer.py:105-113)
__global__ __launch_bounds__(256) void sgd_kernel(long n, float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ buf, float lr, float mom, float wd,
                                                  int has_buf) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float d = g[i] + wd * p[i];
    const float bb = has_buf ? mom * buf[i] + d : d;
    buf[i] = bb;
    p[i] -= lr * bb;
  }
}

// One launch for every parameter of a group (the prompt learner's ctx + Meta-Net: five launches
// at the reference's batch of 1, each a kernel boundary on the step's critical path): tensor
// blockIdx.y, the per-element arithmetic of sgd_kernel (bitwise the same update)
constexpr int kSgdMaxTensors = 16;
struct SgdTensors {
  float* p[kSgdMaxTensors];
  const float* g[kSgdMaxTensors];
  float* buf[kSgdMaxTensors];
  long n[kSgdMaxTensors];
  int has[kSgdMaxTensors];
};
// gs (clipk_sgd_step_multi_scaled): the gradient scale, e.g. the 1 / world of a SUM all-reduce
// (dist.allreduce_grads folds its average here instead of a separate division launch); 1.0 is
// bitwise the unscaled update
// guard (clipk_sgd_step_multi_if): the whole update is skipped when guard[0] & mask != 0 -- the
// PREC fp32s backward's overflow flag, read on the device so the host need not wait for the
// backward before queueing the step (a skipped step leaves p and buf untouched)
template <bool SCALED>
__global__ __launch_bounds__(256) void sgd_multi_kernel(SgdTensors t, float lr, float mom, float wd, float gs,
                                                        const int* __restrict__ guard, int mask) {
  if (guard && (guard[0] & mask)) return;
  const int k = blockIdx.y;
  const long n = t.n[k];
  float* __restrict__ p = t.p[k];
  const float* __restrict__ g = t.g[k];
  float* __restrict__ buf = t.buf[k];
  const int has_buf = t.has[k];
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    // d = fma(wd, p, g) spelled out (the form hipcc contracts the unscaled update to), with the
    // scaled gradient rounded on its own: a power-of-two scale is bitwise the update on
    // pre-scaled gradients
    const float d = __builtin_fmaf(wd, p[i], SCALED ? __fmul_rn(g[i], gs) : g[i]);
    const float bb = has_buf ? mom * buf[i] + d : d;
    buf[i] = bb;
    p[i] -= lr * bb;
  }
}

// clipk_status_take: the status word handed to host-visible memory and cleared, one thread
__global__ __launch_bounds__(64) void status_take_kernel(int* __restrict__ flags, int* __restrict__ host) {
  if (threadIdx.x == 0) {
    const int v = atomicExch(flags, 0);  // (a concurrent stream's OR is never lost between read and clear)
    host[0] = v;
    __threadfence_system();
  }
}

template <typename TO>
__global__ __launch_bounds__(256) void cast_kernel(long n, const float* __restrict__ x, TO* __restrict__ y) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) y[i] = (TO)x[i];
}

// ---------------------------------------------------------------- row gather / scatter
// dst row (dst_rows ? dst_rows[i] : i) = src row (src_rows ? src_rows[i] : i), 16 B per thread
__global__ __launch_bounds__(256) void rows_copy_kernel(int n, int chunks, const uint4* __restrict__ src,
                                                        const int* __restrict__ src_rows, uint4* __restrict__ dst,
                                                        const int* __restrict__ dst_rows) {
  const long total = (long)n * chunks;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int r = (int)(i / chunks), c = (int)(i % chunks);
    const long sr = src_rows ? src_rows[r] : r, dr = dst_rows ? dst_rows[r] : r;
    dst[dr * chunks + c] = src[sr * chunks + c];
  }
}

// Deep prompts (model.py:232-252 IVLP, 293-328 MaPLe): the rows a layer's learnable tokens
// replace. rows[p * n_per + i] = the i-th row that takes prompt row p.
template <typename TD>
__global__ __launch_bounds__(256) void rows_inject_kernel(int n_ctx, int n_per, int W, const float* __restrict__ src,
                                                          const int* __restrict__ rows, TD* __restrict__ dst,
                                                          int ldd) {
  const long total = (long)n_ctx * n_per * W;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int c = (int)(e % W);
    const long ri = e / W;
    const int p = (int)(ri / n_per);
    dst[(size_t)rows[ri] * ldd + c] = (TD)src[(size_t)p * W + c];
  }
}
// out[p] (+)= sum_i src[rows[p*n_per+i]] (fixed order), then those rows of src (and of src2,
// when given) are zeroed: the replaced rows' inputs did not reach the layer.
template <typename TS, typename TS2>
__global__ __launch_bounds__(256) void rows_collect_kernel(int n_ctx, int n_per, int W, TS* __restrict__ src, int lds,
                                                           TS2* __restrict__ src2, int lds2,
                                                           const int* __restrict__ rows, float* __restrict__ out,
                                                           int accumulate, int zero_src) {
  const int p = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (p >= n_ctx || c >= W) return;
  float acc = accumulate ? out[(size_t)p * W + c] : 0.f;
  for (int i = 0; i < n_per; ++i) {
    const size_t r = (size_t)rows[(size_t)p * n_per + i];
    acc += (float)src[r * lds + c];
  }
  out[(size_t)p * W + c] = acc;
  if (zero_src) {
    for (int i = 0; i < n_per; ++i) {
      const size_t r = (size_t)rows[(size_t)p * n_per + i];
      src[r * lds + c] = (TS)0.f;
      if (src2) src2[r * lds2 + c] = (TS2)0.f;
    }
  }
}

static inline int grid_for(long n) {
  long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace clipk

using namespace clipk;

extern "C" int clipk_im2col(int out_dtype, int B, int res, int patch, int Kp, const float* img,
                            void* out, void* stream) {
  if (!img || !out) return CLIPK_EINVAL;
  if (B < 0 || patch <= 0 || res % patch || Kp < 3 * patch * patch) return CLIPK_ESHAPE;
  const long total = (long)B * (res / patch) * (res / patch) * Kp;
  if (total == 0) return CLIPK_OK;
  hipStream_t st = (hipStream_t)stream;
  const int grid = grid_for(total);
  switch (out_dtype) {
    case CLIPK_F16: hipLaunchKernelGGL(im2col_kernel<f16>, grid, 256, 0, st, B, res, patch, Kp, img, (f16*)out); break;
    case CLIPK_BF16: hipLaunchKernelGGL(im2col_kernel<bf16>, grid, 256, 0, st, B, res, patch, Kp, img, (bf16*)out); break;
    case CLIPK_F32: hipLaunchKernelGGL(im2col_kernel<float>, grid, 256, 0, st, B, res, patch, Kp, img, (float*)out); break;
    default: return CLIPK_EDTYPE;
  }
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_vit_embed_ln(int B, int L, int width, const float* patch, const float* cls,
                                  const float* pos, const float* gamma, const float* beta, float* x,
                                  void* stream) {
  if (!patch || !cls || !pos || !gamma || !beta || !x) return CLIPK_EINVAL;
  if (B < 0 || L < 2 || width % 4 || width > 1024) return CLIPK_ESHAPE;
  if (B == 0) return CLIPK_OK;
  hipLaunchKernelGGL(vit_embed_ln_kernel, dim3((B * L + 3) / 4), dim3(256), 0, (hipStream_t)stream, B,
                     L, 0, width, patch, cls, pos, nullptr, gamma, beta, x);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_vit_embed_ln_vpt(int B, int L, int n_vpt, int width, const float* patch, const float* cls,
                                      const float* pos, const float* vpt, const float* gamma, const float* beta,
                                      float* x, void* stream) {
  if (!patch || !cls || !pos || !gamma || !beta || !x || (n_vpt > 0 && !vpt)) return CLIPK_EINVAL;
  if (B < 0 || L < 2 || n_vpt < 0 || width % 4 || width > 1024) return CLIPK_ESHAPE;
  if (B == 0) return CLIPK_OK;
  hipLaunchKernelGGL(vit_embed_ln_kernel, dim3((B * (L + n_vpt) + 3) / 4), dim3(256), 0, (hipStream_t)stream, B,
                     L, n_vpt, width, patch, cls, pos, vpt, gamma, beta, x);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_prompt_assemble(int B, int C, int L, int W, const int* src_map,
                                     const float* emb, const float* ctx, long ctx_sb, long ctx_sc,
                                     const float* bias, const float* pos, float* x0, void* stream) {
  if (!src_map || !emb || !ctx || !pos || !x0) return CLIPK_EINVAL;
  if (B < 0 || C < 0 || L <= 0 || L > 77 || W % 4) return CLIPK_ESHAPE;
  const long rows = (long)B * C * L;
  if (rows == 0) return CLIPK_OK;
  hipLaunchKernelGGL(prompt_assemble_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     B, C, L, W, src_map, emb, ctx, ctx_sb, ctx_sc, bias, pos, x0);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_ctx_grad(int B, int C, int L, int W, int n_ctx, int csc, const int* ctx_pos,
                              const float* dx0, float* dctx, void* stream) {
  if (!ctx_pos || !dx0 || !dctx) return CLIPK_EINVAL;
  if (B <= 0 || C <= 0 || L <= 0 || n_ctx <= 0 || W <= 0) return CLIPK_ESHAPE;
  const int outs = (csc ? B * C : B) * n_ctx;
  hipLaunchKernelGGL(ctx_grad_kernel, dim3(outs, (W + 63) / 64), dim3(256), 0, (hipStream_t)stream, B,
                     C, L, W, n_ctx, csc, ctx_pos, dx0, dctx);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_prompt_assemble_rows(int G, int R, int C, int L, int W, const int* row_tab,
                                          const int* src_map, const float* emb, const float* ctx,
                                          long ctx_sg, long ctx_sc, const float* bias, const float* pos,
                                          float* x0, void* stream) {
  if (!row_tab || !src_map || !emb || !ctx || !pos || !x0) return CLIPK_EINVAL;
  if (G < 0 || R < 0 || C <= 0 || L <= 0 || L > 77 || W % 4) return CLIPK_ESHAPE;
  const long rows = (long)G * R;
  if (rows == 0) return CLIPK_OK;
  hipLaunchKernelGGL(prompt_assemble_rows_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     G, R, L, W, row_tab, src_map, emb, ctx, ctx_sg, ctx_sc, bias, pos, x0);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_ctx_grad_rows(int G, int R, int W, int n_ctx, const int* slot_ptr,
                                   const int* slot_rows, const float* dx0, float* dctx, void* stream) {
  if (!slot_ptr || !slot_rows || !dx0 || !dctx) return CLIPK_EINVAL;
  if (G <= 0 || R <= 0 || n_ctx <= 0 || W <= 0) return CLIPK_ESHAPE;
  hipLaunchKernelGGL(ctx_grad_rows_kernel, dim3(G * n_ctx, (W + 63) / 64), dim3(256), 0, (hipStream_t)stream,
                     R, W, n_ctx, slot_ptr, slot_rows, dx0, dctx);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_cosine_logits_fwd(int B, int C, int E, int per_image, float scale,
                                       const float* imf, const float* txt, float* logits,
                                       float* inv_tnorm, float* inv_inorm, void* stream) {
  if (!imf || !txt || !logits) return CLIPK_EINVAL;
  if (B < 0 || C < 0 || E % 4 || E > 1024) return CLIPK_ESHAPE;
  const long pairs = (long)B * C;
  if (pairs == 0) return CLIPK_OK;
  hipLaunchKernelGGL(cos_logits_fwd_kernel, dim3((pairs + 3) / 4), dim3(256), 0, (hipStream_t)stream, B,
                     C, E, per_image, scale, imf, txt, logits, inv_tnorm, inv_inorm);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_cosine_logits_bwd(int B, int C, int E, int per_image, float scale,
                                       const float* imf, const float* txt, const float* inv_tnorm,
                                       const float* inv_inorm, const float* dlogits, float* dtxt,
                                       void* stream) {
  if (!imf || !txt || !inv_tnorm || !inv_inorm || !dlogits || !dtxt) return CLIPK_EINVAL;
  if (B < 0 || C < 0 || E > 1024) return CLIPK_ESHAPE;
  const long rows = per_image ? (long)B * C : C;
  if (rows == 0) return CLIPK_OK;
  hipLaunchKernelGGL(cos_logits_bwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, B,
                     C, E, per_image, scale, imf, txt, inv_tnorm, inv_inorm, dlogits, dtxt);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_ce_loss(int B, int C, const float* logits, const int64_t* labels,
                             const float* alpha, float gamma, int focal, float grad_scale,
                             float* row_loss, float* dlogits, void* stream) {
  if (!logits || !labels) return CLIPK_EINVAL;
  if (B < 0 || C <= 0) return CLIPK_ESHAPE;
  if (B == 0) return CLIPK_OK;
  hipLaunchKernelGGL(ce_loss_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, B, C, logits, labels,
                     alpha, gamma, focal, grad_scale, row_loss, dlogits);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

static int meta_net_fwd_launch(bool norm, int B, int V, int Hd, int Wd, const float* x, const float* w1,
                               const float* b1, const float* w2, const float* b2, float* xn, float* h, float* y,
                               void* stream) {
  if (!x || !w1 || !b1 || !w2 || !b2 || !y || (norm && !xn)) return CLIPK_EINVAL;
  if (B < 0 || V <= 0 || Hd <= 0 || Wd <= 0) return CLIPK_ESHAPE;
  if (B == 0) return CLIPK_OK;
  hipStream_t st = (hipStream_t)stream;
  if (V % 256 || V > 1024 || Hd > 64 || ((uintptr_t)x | (uintptr_t)w1 | (uintptr_t)xn) % 16) {
    if (norm)
      hipLaunchKernelGGL(meta_net_fwd_generic_kernel<true>, dim3(B), dim3(256), Hd * sizeof(float), st, V, Hd, Wd, x,
                         w1, b1, w2, b2, xn, h, y);
    else
      hipLaunchKernelGGL(meta_net_fwd_generic_kernel<false>, dim3(B), dim3(256), Hd * sizeof(float), st, V, Hd, Wd, x,
                         w1, b1, w2, b2, xn, h, y);
    CLIPK_CHECK_LAUNCH();
    return CLIPK_OK;
  }
  if (norm)
    hipLaunchKernelGGL(meta_net_fwd_kernel<true>, dim3(B, (Wd + 63) / 64), dim3(256), Hd * sizeof(float), st, V, Hd,
                       Wd, x, w1, b1, w2, b2, xn, h, y);
  else
    hipLaunchKernelGGL(meta_net_fwd_kernel<false>, dim3(B, (Wd + 63) / 64), dim3(256), Hd * sizeof(float), st, V, Hd,
                       Wd, x, w1, b1, w2, b2, xn, h, y);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_meta_net_fwd(int B, int V, int Hd, int Wd, const float* x, const float* w1,
                                  const float* b1, const float* w2, const float* b2, float* h,
                                  float* y, void* stream) {
  return meta_net_fwd_launch(false, B, V, Hd, Wd, x, w1, b1, w2, b2, nullptr, h, y, stream);
}

extern "C" int clipk_meta_net_fwd_norm(int B, int V, int Hd, int Wd, const float* x, const float* w1,
                                       const float* b1, const float* w2, const float* b2, float* xn, float* h,
                                       float* y, void* stream) {
  return meta_net_fwd_launch(true, B, V, Hd, Wd, x, w1, b1, w2, b2, xn, h, y, stream);
}

extern "C" int clipk_ce_loss_reduce(int B, int C, const float* logits, const int64_t* labels, const float* alpha,
                                    float gamma, int focal, float grad_scale, int reduction, float* row_loss,
                                    float* loss, float* dlogits, void* stream) {
  if (!logits || !labels || !row_loss || !loss) return CLIPK_EINVAL;
  if (reduction != 1 && reduction != 2) return CLIPK_EINVAL;
  if (B <= 0 || C <= 0) return CLIPK_ESHAPE;
  hipLaunchKernelGGL(ce_loss_reduce_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, B, C, logits, labels, alpha,
                     gamma, focal, grad_scale, reduction == 1 ? 1 : 0, row_loss, loss, dlogits);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_ctx_bias_grad_rows(int G, int R, int W, int n_ctx, const int* slot_ptr, const int* slot_rows,
                                        const float* dx0, float* dctx, float* dbias, void* stream) {
  if (!slot_ptr || !slot_rows || !dx0 || !dctx) return CLIPK_EINVAL;
  if (G <= 0 || R <= 0 || n_ctx <= 0 || W <= 0) return CLIPK_ESHAPE;
  hipLaunchKernelGGL(ctx_bias_grad_rows_kernel, dim3((W + 255) / 256), dim3(256), 0, (hipStream_t)stream, G, R, W,
                     n_ctx, slot_ptr, slot_rows, dx0, dctx, dbias);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_status_take(int* flags, int* host_word, void* stream) {
  if (!flags || !host_word) return CLIPK_EINVAL;
  hipLaunchKernelGGL(status_take_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, flags, host_word);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_meta_net_bwd(int B, int V, int Hd, int Wd, const float* x, const float* h,
                                  const float* w2, const float* dy, float* dw1, float* db1,
                                  float* dw2, float* db2, float* dh_ws, void* stream) {
  if (!x || !h || !w2 || !dy || !dw1 || !db1 || !dw2 || !db2 || !dh_ws) return CLIPK_EINVAL;
  if (B <= 0 || V <= 0 || Hd <= 0 || Wd <= 0) return CLIPK_ESHAPE;
  hipStream_t st = (hipStream_t)stream;
  const int nb_dh = (B * Hd + 3) / 4;
  const long nw2 = (long)Wd * Hd, nw1 = (long)Hd * V;
  hipLaunchKernelGGL(meta_net_bwd_a_kernel, dim3(nb_dh + (nw2 + 255) / 256), dim3(256), 0, st, B, Hd, Wd, nb_dh,
                     h, w2, dy, dw2, db2, dh_ws);
  CLIPK_CHECK_LAUNCH();
  hipLaunchKernelGGL(meta_net_bwd_b_kernel, dim3((nw1 + 255) / 256), dim3(256), 0, st, B, V, Hd, x, dh_ws, dw1,
                     db1);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

static int sgd_multi(int count, float* const* p, const float* const* g, float* const* buf, const long* n,
                     const int* has_buf, float lr, float momentum, float weight_decay, float grad_scale,
                     const int* guard, int mask, void* stream);

extern "C" int clipk_sgd_step_multi(int count, float* const* p, const float* const* g, float* const* buf,
                                    const long* n, const int* has_buf, float lr, float momentum,
                                    float weight_decay, void* stream) {
  return sgd_multi(count, p, g, buf, n, has_buf, lr, momentum, weight_decay, 1.0f, nullptr, 0, stream);
}

extern "C" int clipk_sgd_step_multi_scaled(int count, float* const* p, const float* const* g, float* const* buf,
                                           const long* n, const int* has_buf, float lr, float momentum,
                                           float weight_decay, float grad_scale, void* stream) {
  return sgd_multi(count, p, g, buf, n, has_buf, lr, momentum, weight_decay, grad_scale, nullptr, 0, stream);
}

extern "C" int clipk_sgd_step_multi_if(int count, float* const* p, const float* const* g, float* const* buf,
                                       const long* n, const int* has_buf, float lr, float momentum,
                                       float weight_decay, float grad_scale, const int* guard, int mask,
                                       void* stream) {
  if (!guard) return CLIPK_EINVAL;
  return sgd_multi(count, p, g, buf, n, has_buf, lr, momentum, weight_decay, grad_scale, guard, mask, stream);
}

static int sgd_multi(int count, float* const* p, const float* const* g, float* const* buf, const long* n,
                     const int* has_buf, float lr, float momentum, float weight_decay, float grad_scale,
                     const int* guard, int mask, void* stream) {
  if (count < 0 || count > kSgdMaxTensors || (count && (!p || !g || !buf || !n || !has_buf))) return CLIPK_EINVAL;
  SgdTensors t{};
  long nmax = 0;
  for (int k = 0; k < count; ++k) {
    if (!p[k] || !g[k] || !buf[k]) return CLIPK_EINVAL;
    if (n[k] < 0) return CLIPK_ESHAPE;
    t.p[k] = p[k];
    t.g[k] = g[k];
    t.buf[k] = buf[k];
    t.n[k] = n[k];
    t.has[k] = has_buf[k];
    nmax = n[k] > nmax ? n[k] : nmax;
  }
  if (nmax == 0) return CLIPK_OK;
  if (grad_scale == 1.0f)
    hipLaunchKernelGGL(sgd_multi_kernel<false>, dim3(grid_for(nmax), count), dim3(256), 0, (hipStream_t)stream, t, lr,
                       momentum, weight_decay, 1.0f, guard, mask);
  else
    hipLaunchKernelGGL(sgd_multi_kernel<true>, dim3(grid_for(nmax), count), dim3(256), 0, (hipStream_t)stream, t, lr,
                       momentum, weight_decay, grad_scale, guard, mask);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_sgd_step(long n, float* p, const float* g, float* buf, float lr,
                              float momentum, float weight_decay, int has_buf, void* stream) {
  if (!p || !g || !buf) return CLIPK_EINVAL;
  if (n < 0) return CLIPK_ESHAPE;
  if (n == 0) return CLIPK_OK;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, n, p, g, buf, lr,
                     momentum, weight_decay, has_buf);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_rows_copy(int row_bytes, int n, const void* src, const int* src_rows, void* dst,
                               const int* dst_rows, void* stream) {
  if (!src || !dst) return CLIPK_EINVAL;
  if (n < 0 || row_bytes <= 0 || row_bytes % 16) return CLIPK_ESHAPE;
  if (((uintptr_t)src | (uintptr_t)dst) & 15) return CLIPK_ESHAPE;
  if (n == 0) return CLIPK_OK;
  const int chunks = row_bytes / 16;
  hipLaunchKernelGGL(rows_copy_kernel, grid_for((long)n * chunks), 256, 0, (hipStream_t)stream, n, chunks,
                     (const uint4*)src, src_rows, (uint4*)dst, dst_rows);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_rows_inject(int dst_dtype, int n_ctx, int n_per, int width, const float* src, const int* rows,
                                 void* dst, int ldd, void* stream) {
  if (!src || !rows || !dst) return CLIPK_EINVAL;
  if (n_ctx < 0 || n_per < 0 || width <= 0 || ldd < width) return CLIPK_ESHAPE;
  const long total = (long)n_ctx * n_per * width;
  if (total == 0) return CLIPK_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (dst_dtype) {
    case CLIPK_F32: hipLaunchKernelGGL(rows_inject_kernel<float>, grid_for(total), 256, 0, st, n_ctx, n_per, width, src, rows, (float*)dst, ldd); break;
    case CLIPK_F16: hipLaunchKernelGGL(rows_inject_kernel<f16>, grid_for(total), 256, 0, st, n_ctx, n_per, width, src, rows, (f16*)dst, ldd); break;
    case CLIPK_BF16: hipLaunchKernelGGL(rows_inject_kernel<bf16>, grid_for(total), 256, 0, st, n_ctx, n_per, width, src, rows, (bf16*)dst, ldd); break;
    default: return CLIPK_EDTYPE;
  }
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_rows_collect(int src_dtype, int n_ctx, int n_per, int width, void* src, int lds, void* src2,
                                  int src2_dtype, int lds2, const int* rows, float* out, int accumulate,
                                  int zero_src, void* stream) {
  if (!src || !rows || !out) return CLIPK_EINVAL;
  if (n_ctx < 0 || n_per < 0 || width <= 0 || lds < width || (src2 && lds2 < width)) return CLIPK_ESHAPE;
  if (n_ctx == 0) return CLIPK_OK;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((width + 255) / 256, n_ctx);
  auto go = [&](auto* s1) {
    using TS = std::remove_pointer_t<decltype(s1)>;
    if (!src2) {
      hipLaunchKernelGGL((rows_collect_kernel<TS, float>), grid, 256, 0, st, n_ctx, n_per, width, s1, lds,
                         (float*)nullptr, 0, rows, out, accumulate, zero_src);
      return CLIPK_OK;
    }
    switch (src2_dtype) {
      case CLIPK_F32: hipLaunchKernelGGL((rows_collect_kernel<TS, float>), grid, 256, 0, st, n_ctx, n_per, width, s1, lds, (float*)src2, lds2, rows, out, accumulate, zero_src); break;
      case CLIPK_F16: hipLaunchKernelGGL((rows_collect_kernel<TS, f16>), grid, 256, 0, st, n_ctx, n_per, width, s1, lds, (f16*)src2, lds2, rows, out, accumulate, zero_src); break;
      case CLIPK_BF16: hipLaunchKernelGGL((rows_collect_kernel<TS, bf16>), grid, 256, 0, st, n_ctx, n_per, width, s1, lds, (bf16*)src2, lds2, rows, out, accumulate, zero_src); break;
      default: return CLIPK_EDTYPE;
    }
    return CLIPK_OK;
  };
  int rc;
  switch (src_dtype) {
    case CLIPK_F32: rc = go((float*)src); break;
    case CLIPK_F16: rc = go((f16*)src); break;
    case CLIPK_BF16: rc = go((bf16*)src); break;
    default: return CLIPK_EDTYPE;
  }
  if (rc != CLIPK_OK) return rc;
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

extern "C" int clipk_cast(int out_dtype, long n, const float* x, void* y, void* stream) {
  if (!x || !y) return CLIPK_EINVAL;
  if (n <= 0) return n == 0 ? CLIPK_OK : CLIPK_ESHAPE;
  hipStream_t st = (hipStream_t)stream;
  switch (out_dtype) {
    case CLIPK_F16: hipLaunchKernelGGL(cast_kernel<f16>, grid_for(n), 256, 0, st, n, x, (f16*)y); break;
    case CLIPK_BF16: hipLaunchKernelGGL(cast_kernel<bf16>, grid_for(n), 256, 0, st, n, x, (bf16*)y); break;
    case CLIPK_F32: hipLaunchKernelGGL(cast_kernel<float>, grid_for(n), 256, 0, st, n, x, (float*)y); break;
    default: return CLIPK_EDTYPE;
  }
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}
