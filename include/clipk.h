/*
 * clipk.h — C-ABI of the MI355X-native CoOp/CoCoOp hot path (libclipk.so).
 *
 * Plain pointers + sizes + a hipStream_t (passed as void*); no torch types.
 * Every device pointer is owned by the caller (the torch caching allocator in
 * the Python host). Kernels never allocate. Encoder handles hold only HOST-side
 * pointer tables to caller-owned, packed, frozen weights.
 *
 * Return value: CLIPK_OK (0); a negative CLIPK_E* for bad arguments (checked on
 * the host BEFORE any launch); a positive hipError_t from a failed launch.
 *
 * Reference interfaces replaced (PyTorch ops inside the reference hot path):
 *   clipk_gemm            nn.Linear / MHA in_proj,out_proj / mlp.c_fc,c_proj / @proj
 *                         (PromptSRC/clip/model.py:171-177, 429; trainers/coop.py:204)
 *   clipk_layernorm_*     LayerNorm (model.py:153-159) fwd / input-grad bwd
 *   clipk_attention_*     nn.MultiheadAttention SDPA core (model.py:181-183, mask 592-598)
 *   clipk_im2col          VisionTransformer.conv1 patch embed as GEMM (model.py:376,402)
 *   clipk_vit_embed_ln    cls cat + pos add + ln_pre (model.py:405-420)
 *   clipk_prompt_assemble PromptLearner.forward cat + TextEncoder pos add
 *                         (trainers/coop.py:259-296, cocoop.py:173-198, coop.py:197)
 *   clipk_ctx_grad        autograd of that cat w.r.t. ctx (coop.py:265, cocoop.py:186-194)
 *   clipk_cosine_logits_* CustomCLIP normalize + logit_scale.exp() * imf @ txt^T
 *                         (coop.py:356-363, cocoop.py:238-251)
 *   clipk_ce_loss         nn.CrossEntropyLoss / MultiClassFocalLoss fwd+bwd
 *                         (coop.py:131-163,324; cocoop.py:66-101,233)
 *   clipk_meta_net_*      CoCoOp Meta-Net Linear-ReLU-Linear (cocoop.py:139-143,182-185)
 *   clipk_sgd_step        torch.optim.SGD momentum/wd step (dassl optim/optimizer.py:105-113)
 *   clipk_sgd_step_multi  the same over a param group's tensors in one launch
 *   clipk_text_*          TextEncoder.forward + its input-grad backward (coop.py:195-205)
 *   clipk_vit_forward     VisionTransformer.forward (model.py:401-431), frozen, fwd only
 */
#ifndef CLIPK_H
#define CLIPK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* element types. CLIPK_F32S (GEMM input type only): fp32 activations times a weight packed by
 * clipk_split_pack -- the fp32-class GEMM on 16-bit MFMA of PREC "fp32s" (clipk_gemm).
 * CLIPK_F32S16 (GEMM input type only): the same product for an fp16-valued weight (every lo part
 * of its clipk_split_pack output zero, as for every released CLIP checkpoint -- the reference
 * loads them from the fp16 archive, PromptSRC/clip/clip.py:154-180), whose B operand is the
 * COMPACT weight of clipk_split_hi16: fp16 [N, K] = CLIPK_SPLIT_SCALE * W exactly, 2 B per element
 * (ldb == K). The hi(a) lo(b) product, exactly zero, is not formed: 2 MFMAs per product instead of
 * 3, and half of B's bytes staged; results bitwise those of CLIPK_F32S on the packed weight. */
enum { CLIPK_F32 = 0, CLIPK_F16 = 1, CLIPK_BF16 = 2, CLIPK_F32S = 3, CLIPK_F32S16 = 4 };

/* status codes (hipError_t values > 0 pass through) */
enum {
  CLIPK_OK = 0,
  CLIPK_EINVAL = -1,     /* null pointer / bad enum */
  CLIPK_ESHAPE = -2,     /* shape violates a kernel constraint */
  CLIPK_EDTYPE = -3,     /* unsupported dtype combination */
  CLIPK_EWORKSPACE = -4, /* workspace too small */
  CLIPK_ERANGE = -5,     /* an input outside the range the kernel supports (clipk_split_pack,
                            clipk_split_hi16) */
  CLIPK_EHIP = -6        /* a HIP runtime call of a synchronous check failed (clipk_split_*) */
};

/* GEMM epilogues:  acc = A[M,K] . B[N,K]^T  (fp32 accumulate)                         */
enum {
  CLIPK_EPI_BIAS = 0,       /* out(out_dtype) = acc + bias                                */
  CLIPK_EPI_BIAS_RES = 1,   /* out = acc + bias + res; out and res both f32, or both the
                               16-bit in_dtype (16-bit residual stream)                  */
  CLIPK_EPI_BIAS_QGELU = 2, /* out = quickgelu(acc + bias); out2 (optional) = acc + bias */
  CLIPK_EPI_DQGELU = 3,     /* out = acc * quickgelu'(aux)                                */
  CLIPK_EPI_NONE = 4        /* out = acc                                                  */
};
/* Operand flag OR-ed into epi: A is a pre-activation h and the GEMM consumes quickgelu(h)
 * (applied to each 16-B chunk of A as it is staged into LDS), so the producer of h need
 * not also write quickgelu(h) (the text c_proj forward). 16-bit in_dtype only. */
enum { CLIPK_A_QGELU = 0x100 };
/* Epilogue flag OR-ed into epi, training's QuickGELU pair (replaces keeping the pre-activation,
 * PromptSRC/clip/model.py:162-164, 177): with CLIPK_EPI_BIAS_QGELU, out2 = quickgelu'(acc + bias)
 * instead of acc + bias; with CLIPK_EPI_DQGELU, aux already holds quickgelu'(h) and
 * out = acc * aux. The forward epilogue has sigmoid(1.702 h) in hand (three more VALU per element);
 * the backward epilogue drops its exp + rcp per element. Also accepted by clipk_gemm_ln (fold
 * form of EPI_BIAS_QGELU) and clipk_gemm_splitk (EPI_BIAS_QGELU). */
enum { CLIPK_QGELU_DERIV = 0x200 };
/* PREC fp32s operand flags OR-ed into epi (split in_dtype CLIPK_F32S / CLIPK_F32S16, fp32 out).
 * The split GEMM forms each activation's fp16 parts hi = fp16(x), lo = fp16(x - hi) itself; a
 * PRE-SPLIT operand holds them already: [rows, K] 4-byte elements, per 8 consecutive k 16 B of hi
 * parts then 16 B of lo parts (clipk_split_pack's layout at scale 1).
 *  CLIPK_OUT_SPLIT: out is stored pre-split (the fp32 result's parts; for the next GEMM's A).
 *    clipk_gemm (EPI_BIAS_QGELU [| QGELU_DERIV], EPI_DQGELU | QGELU_DERIV) and the folds
 *    clipk_gemm_ln / clipk_gemm_ln_gamma (c_fc).
 *  CLIPK_A_SPLIT: A is given pre-split, as such a producer wrote it; the GEMM forms no split.
 *    clipk_gemm (EPI_NONE, EPI_BIAS_RES, EPI_DQGELU | QGELU_DERIV), the producer form of
 *    clipk_gemm_ln, clipk_gemm_ln_gamma (A = the split parts of x * gamma, which the call then
 *    does not apply again: clipk_gemm_ln_stats_split writes them) and clipk_gemm_ln_stats_split.
 *  (CLIPK_OUT2_SPLIT_GAMMA: internal to clipk_gemm_ln_stats_split.)
 * Results are bitwise those of the same GEMMs on the fp32 values: the parts are the ones the GEMM
 * would form (PREC fp32s: the split VALU leaves the K loop's critical path). */
enum { CLIPK_OUT_SPLIT = 0x400, CLIPK_A_SPLIT = 0x800, CLIPK_OUT2_SPLIT_GAMMA = 0x1000 };

const char* clipk_version(void);
/* sha256 (hex) over the sources this library was built from: csrc/{*.hip,*.h,Makefile} and
 * include/clipk.h, in file-name order, each as "<sha256 of content>  <relative path>\n"
 * (fsp_amd/_native.py source_digest; the loader refuses a library built from another tree). */
const char* clipk_source_digest(void);
const char* clipk_strerror(int status);
int clipk_device_arch_ok(void); /* 1 if device 0 is gfx950 */

/* ---------------------------------------------------------------- primitives */
/* Constraints: N % 128 == 0, K % 64 == 0 (16-bit) or K % 32 == 0 (f32); lda,ldb,ldo
 * multiples of 8 elements; A/B of in_dtype; bias/res fp32; aux of aux_dtype. */
int clipk_gemm(int in_dtype, int out_dtype, int epi, int M, int N, int K,
               const void* A, int lda, const void* B, int ldb,
               const float* bias, const void* res, int ldr,
               void* out, int ldo, void* out2, const void* aux, int aux_dtype, int ldaux,
               void* stream);

/* fp32-class GEMM on the 16-bit MFMA (PREC "fp32s"; the reference runs these Linear layers in
 * fp32, PromptSRC/clip/model.py:171-177, 699). clipk_split_pack stores W [N, K] (fp32, row
 * stride ldw) as CLIPK_SPLIT_SCALE * W split into fp16 parts hi = fp16(x), lo = fp16(x - hi):
 * per 8 consecutive k, 16 B of hi then 16 B of lo (4 B per element, the out buffer holds
 * N * K * 4 bytes; K % 32 == 0). |W| must stay below 65504 / CLIPK_SPLIT_SCALE: the call
 * checks it (one pass over W, then a stream synchronisation: packing runs once per model) and
 * returns CLIPK_ERANGE for a larger or non-finite value. clipk_gemm(in_dtype = CLIPK_F32S, ...)
 * then takes A fp32 [M, K] and B = the packed weight (ldb must equal K) and forms every product as hi(a) hi(b) + hi(a) lo(b) + lo(a) hi(b) with
 * v_mfma_f32_16x16x32_f16 (fp32 accumulate; A split in registers as its fragments are read),
 * scaled by 1 / CLIPK_SPLIT_SCALE before the epilogue: ~22 significant bits per operand, the
 * fp32 result to ~1e-6 relative. out / res / aux fp32 (epilogues as above). */
#define CLIPK_SPLIT_SCALE 64.0f
int clipk_split_pack(int N, int K, const float* W, int ldw, void* out, void* stream);
/* *result = 1 when every lo part of clipk_split_pack's output `packed` ([N, K] split elements) is
 * zero (the weight is fp16-valued: clipk_split_hi16 may compact it for CLIPK_F32S16), 0 when not.
 * Returns CLIPK_OK, or a negative status (CLIPK_EHIP for a failed HIP call; *result untouched).
 * One pass, then a stream synchronisation (checked once per weight, at model construction). */
int clipk_split_lo_zero(int N, int K, const void* packed, int* result, void* stream);
/* The CLIPK_F32S16 B operand: out fp16 [N, K] = the hi parts of clipk_split_pack's output `packed`
 * (= CLIPK_SPLIT_SCALE * W exactly). CLIPK_ERANGE when a lo part is nonzero (W is not fp16-valued;
 * out is then unspecified). One pass, then a stream synchronisation. */
int clipk_split_hi16(int N, int K, const void* packed, void* out, void* stream);

/* Split-K form of clipk_gemm for small M (the ViT at training batch sizes, whose 128x128
 * tile grid would leave most CUs idle): the K range is cut into `splits` slices whose fp32
 * partials go to the caller's workspace ws ([splits][M][N] fp32), then one elementwise pass
 * sums them in slice order (deterministic) and applies the epilogue. Same arguments and
 * epilogues as clipk_gemm except EPI_DQGELU; splits <= 0 picks clipk_gemm_auto_splits;
 * one slice is plain clipk_gemm (ws unused). */
int clipk_gemm_auto_splits(int in_dtype, int M, int N, int K);
size_t clipk_gemm_splitk_ws_bytes(int M, int N, int splits);
int clipk_gemm_splitk(int in_dtype, int out_dtype, int epi, int M, int N, int K,
                      const void* A, int lda, const void* B, int ldb,
                      const float* bias, const void* res, int ldr,
                      void* out, int ldo, void* out2, int splits, void* ws, size_t ws_bytes,
                      void* stream);

/* LayerNorm folded into the GEMM that consumes it (the text encoder's ln_1 -> attn.in_proj
 * and ln_2 -> mlp.c_fc, PromptSRC/clip/model.py:153-159, 185-188):
 *   LN(x) W^T + b = rstd * (x W'^T - mean * s) + c,  W' = W diag(gamma) (in_dtype),
 *   s_j = sum_k W'[j,k], c_j = b_j + sum_k beta_k W[j,k] (fp32),
 * so the GEMM reads the residual stream x itself and no normalised copy is written.
 * Two modes, 16-bit in_dtype == out dtype, or in_dtype CLIPK_F32S (A, out, res fp32; B = W'
 * split-packed by clipk_split_pack; s summed over the packed value, (hi + lo) / 64):
 *  - colsum == NULL: EPI_BIAS_RES (the residual-stream producer); in addition, per row m and
 *    64-column group g of the ROUNDED output, stats[(m * N/64 + g) * 2 + {0, 1}] = (sum, sum of
 *    squared deviations from the group's mean) (fp32);
 *  - colsum != NULL (stats NULL): EPI_BIAS or EPI_BIAS_QGELU with A = x, B = W', bias = c,
 *    colsum = s and rnb = per-row (rstd, -rstd * mean) pairs of A's rows (fp32 [M][2]).
 * clipk_ln_stats_merge turns a producer's partials (width / 64 per row) into any of mean, rstd
 * (fp32 [rows]) and rnb (exact pairwise merge in a fixed order, eps 1e-5). Shape constraints as
 * clipk_gemm. */
/* The fold with the LayerNorm weight on A (PREC fp32s, in_dtype CLIPK_F32S / CLIPK_F32S16; the
 * consumer form of clipk_gemm_ln): A = x fp32 [M, K] (K <= 1024), B = W packed (ldb == K), each
 * x[m, k] * gamma[k] rounded to fp32 before its split; colsum = rowsums of W diag(gamma) over the
 * packed value / 64 (fp32 [N]), bias = b + W beta, rnb as in clipk_gemm_ln. Keeps an fp16-valued
 * W fp16-valued, so CLIPK_F32S16's 2 MFMAs per product apply to the folded GEMMs too. */
int clipk_gemm_ln_gamma(int in_dtype, int epi, int M, int N, int K, const void* A, int lda, const void* B, int ldb,
                        const float* bias, void* out, int ldo, void* out2, const float* colsum, const float* rnb,
                        const float* gamma, void* stream);
int clipk_gemm_ln(int in_dtype, int epi, int M, int N, int K, const void* A, int lda, const void* B, int ldb,
                  const float* bias, const void* res, int ldr, void* out, int ldo, void* out2,
                  float* stats, const float* colsum, const float* rnb, void* stream);
/* The statistics producer of clipk_gemm_ln (EPI_BIAS_RES [| CLIPK_A_SPLIT], colsum NULL), in_dtype
 * CLIPK_F32S16, that also stores out2 [M, N] = the pre-split form (CLIPK_OUT_SPLIT) of out * gamma,
 * the fp32 products the next fold (clipk_gemm_ln_gamma, gamma = its LayerNorm weight) would form:
 * that fold then reads out2 with CLIPK_A_SPLIT. The residual stream out stays fp32. */
int clipk_gemm_ln_stats_split(int in_dtype, int epi, int M, int N, int K, const void* A, int lda, const void* B,
                              int ldb, const float* bias, const void* res, int ldr, void* out, int ldo, float* stats,
                              const float* gamma, void* out2, void* stream);
int clipk_ln_stats_merge(int rows, int width, const float* stats, float* mean, float* rstd, float* rnb,
                         void* stream);
/* clipk_ln_stats_merge(M, K, stats, mean, rstd, rnb) followed by the fold clipk_gemm_ln(...,
 * colsum, rnb) (res NULL), as ONE launch where the library covers the shape in-kernel (16-bit,
 * K = 512, the 192-row tile configuration: the batch-1 text encoder's LN-fold GEMMs), else as
 * those two calls. Outputs are bitwise those of the two calls: out / out2, mean and rstd
 * (optional) and rnb (required). Replaces the merge launch between a producer and its fold
 * (PromptSRC/clip/model.py:153-159, 185-188: ln_1 / ln_2 of each residual block). */
int clipk_gemm_ln_merge(int in_dtype, int epi, int M, int N, int K, const void* A, int lda, const void* B,
                        int ldb, const float* bias, void* out, int ldo, void* out2, const float* stats,
                        const float* colsum, float* mean, float* rstd, float* rnb, void* stream);
/* 1 when clipk_gemm_ln_merge runs the shape as one launch, 0 when as the two calls. */
int clipk_gemm_ln_merge_fused(int in_dtype, int M, int N, int K);
/* Benchmark knob: force the 16-bit GEMM tile configuration (0: 128x128, 1: 256x256
 * (persistent above 2 x CUs tiles), 2: 256x128, 3: 256x256 non-persistent, 6: 192x256;
 * -1 = automatic by shape; other values: CLIPK_EINVAL). Not needed for normal use. */
int clipk_gemm_set_config(int cfg);

/* Image preprocessing (Dassl/torchvision Resize+CenterCrop / RandomResizedCrop+flip,
 * ToTensor, Normalize; transforms.py:206-354): Pillow-exact bicubic resampling of a crop
 * window of each uint8 HWC image (src: packed images), from host-built fixed-point tables
 * (fsp_amd/data/preprocess.py documents desc/tables); out fp32 [B,3,S,S] normalised with
 * mean/std, or the uint8 pixels when out_uint8. tmp: sum over images of rows*S*3 bytes. */
int clipk_image_resample(int B, int S, int rows_max, const void* src, const long long* desc,
                         const int* tables, void* tmp, const float* mean, const float* stdv,
                         int out_uint8, void* out, void* stream);

/* Diagnostic: per-block / per-tile s_memrealtime marks of the last GEMM launch, recorded
 * only when the process runs with CLIPK_GEMM_STAMP set (synchronises the device). */
int clipk_gemm_stamps(void* host, size_t bytes);

/* cls cat + pos add + ln_pre with n_vpt visual prompt rows appended per image (IVLP / MaPLe /
 * PromptSRC, model.py:413-420, 465-472): x[b*(L+n_vpt) + t] = ln_pre(t < L ? embed(b, t) :
 * vpt[t-L]) (prompts get no positional embedding). */
int clipk_vit_embed_ln_vpt(int B, int L, int n_vpt, int width, const float* patch, const float* cls,
                           const float* pos, const float* vpt, const float* gamma, const float* beta, float* x,
                           void* stream);

/* Deep prompts (ResidualAttentionBlock_IVLP / _MaPLe.forward, model.py:229-256, 287-331): the
 * rows a layer's learnable tokens replace. rows[p*n_per + i] = i-th row taking prompt row p.
 * inject: dst[rows[p*n_per+i]] = (dst dtype) src[p]   (src [n_ctx, width] fp32).
 * collect: out[p] (+= when accumulate) sum_i src[rows[p*n_per+i]] in a fixed order, then those
 * rows of src (and of src2, a second copy of the same stream, when given) are zeroed. */
int clipk_rows_inject(int dst_dtype, int n_ctx, int n_per, int width, const float* src, const int* rows,
                      void* dst, int ldd, void* stream);
int clipk_rows_collect(int src_dtype, int n_ctx, int n_per, int width, void* src, int lds, void* src2,
                       int src2_dtype, int lds2, const int* rows, float* out, int accumulate, int zero_src,
                       void* stream);

/* y = LN(x[row]) for rows r in [0,rows): x row = in_rows ? in_rows[r] : r.
 * out of out_dtype with row stride ldo; mean/rstd (optional, fp32 [rows]). width%64==0, <=1024 */
int clipk_layernorm_fwd(int out_dtype, int rows, int width, const float* x, int ldx,
                        const int* in_rows, const float* gamma, const float* beta,
                        void* out, int ldo, float* mean, float* rstd, void* stream);
/* same with x of x_dtype (fp32 or 16-bit: the 16-bit text residual stream) */
int clipk_layernorm_fwd_x(int x_dtype, int out_dtype, int rows, int width, const void* x, int ldx,
                          const int* in_rows, const float* gamma, const float* beta,
                          void* out, int ldo, float* mean, float* rstd, void* stream);

/* dx = LN-input-grad(dy; x, gamma, mean, rstd) (+ dres). dy of dy_dtype; x row = x_rows ? x_rows[r] : r;
 * outputs written at row out_rows ? out_rows[r] : r of dx (f32) and dx_lp (lp_dtype, optional;
 * lp_dtype CLIPK_F32S: dx_lp in the pre-split form of CLIPK_A_SPLIT, the next split GEMMs' A). */
int clipk_layernorm_bwd(int dy_dtype, int rows, int width, const void* dy, int lddy, const float* x, int ldx,
                        const int* x_rows, const float* gamma, const float* mean, const float* rstd,
                        const float* dres, int lddres, float* dx, void* dx_lp, int lp_dtype,
                        const int* out_rows, int ldo, void* stream);
/* same with x of x_dtype */
int clipk_layernorm_bwd_x(int x_dtype, int dy_dtype, int rows, int width, const void* dy, int lddy,
                          const void* x, int ldx, const int* x_rows, const float* gamma,
                          const float* mean, const float* rstd, const float* dres, int lddres,
                          float* dx, void* dx_lp, int lp_dtype, const int* out_rows, int ldo,
                          void* stream);
/* same with the residual gradient dres of dres_dtype: fp32, or lp_dtype (a 16-bit residual-
 * gradient stream; dres may then alias dx_lp, updated in place). dx (fp32) may be NULL when
 * dx_lp is given. */
int clipk_layernorm_bwd_x2(int x_dtype, int dy_dtype, int rows, int width, const void* dy, int lddy,
                           const void* x, int ldx, const int* x_rows, const float* gamma,
                           const float* mean, const float* rstd, const void* dres, int dres_dtype,
                           int lddres, float* dx, void* dx_lp, int lp_dtype, const int* out_rows,
                           int ldo, void* stream);

/* Multi-head self-attention core on packed qkv rows [(s*L+t), 3*heads*64] (head dim 64):
 * out[(s*L+t), h*64+d]; lse[(s*L+t)*heads + h] (optional) = logsumexp of scaled scores. */
int clipk_attention_fwd(int dtype, int nseq, int L, int heads, int causal,
                        const void* qkv, int ldqkv, void* out, int ldo, float* lse, void* stream);

/* Input-grad backward of the attention core, any L (L <= 16: one MFMA tile; longer: two MFMA
 * passes, dK/dV per key tile and dQ per query tile; VALU for fp32): dqkv (grad_dtype) from qkv
 * and the saved forward output ofwd (dtype), dout (grad_dtype) and lse. */
int clipk_attention_bwd(int dtype, int grad_dtype, int nseq, int L, int heads, int causal,
                        const void* qkv, int ldqkv, const void* ofwd, int ldof, const void* dout,
                        int lddo, const float* lse, void* dqkv, int lddqkv, void* stream);

/* Shared-prefix packed attention (text, causal). Rows of group g (stride R) hold the P
 * prefix rows shared by all sequences of the group, then each sequence's own rows. The
 * class rows are covered in order by ntiles tiles of <= 16 rows holding whole sequences:
 * tiles[2t], tiles[2t+1] = (group-relative first row, rows); row_first[r] (r < R) = first
 * row of the sequence that row r belongs to (0 for prefix rows). A class row attends to all
 * P prefix keys plus the rows of its own sequence causally; the prefix rows attend among
 * themselves causally. 1 <= P <= 16. Exact restatement of the causal attention of the
 * unpacked [C, L] prompts (attention_prefix.hip). */
int clipk_attention_prefix_fwd(int dtype, int G, int P, int R, int ntiles, const int* tiles,
                               const int* row_first, int heads, const void* qkv, int ldqkv, void* out,
                               int ldo, float* lse, void* stream);
/* Backward; ws >= clipk_attention_prefix_ws_bytes(G, ntiles, heads) holds the per-chunk fp32
 * partial dK/dV of the prefix rows (reduced in a fixed order). grad_dtype CLIPK_F32S (dtype
 * CLIPK_F32, PREC fp32s): fp32 dout, dqkv stored in the pre-split form of CLIPK_A_SPLIT (the qkv
 * input-grad GEMM's A; ldqkv % 8 == 0), the parts of the same fp32 values. */
size_t clipk_attention_prefix_ws_bytes(int G, int ntiles, int heads);
int clipk_attention_prefix_bwd(int dtype, int grad_dtype, int G, int P, int R, int ntiles,
                               const int* tiles, const int* row_first, int heads, const void* qkv,
                               int ldqkv, const void* ofwd, int ldof, const void* dout, int lddo,
                               const float* lse, void* dqkv, int lddqkv, void* ws, size_t ws_bytes,
                               void* stream);

/* The same with flags: CLIPK_PREFIX_CLS_GROUP0 -- every group's class rows read their q|k|v from
 * group 0's rows (the text encoder's layer 0, where the class rows enter every group with the
 * same values: clipk_encoder_set_input_rows; rows [P, R) of groups >= 1 of qkv are then never
 * read, so no copies of group 0's are written). Prefix rows, outputs, dout, lse per group. */
enum { CLIPK_PREFIX_CLS_GROUP0 = 1 };
int clipk_attention_prefix_fwd_ex(int dtype, int G, int P, int R, int ntiles, const int* tiles,
                                  const int* row_first, int heads, const void* qkv, int ldqkv, void* out,
                                  int ldo, float* lse, int flags, void* stream);
int clipk_attention_prefix_bwd_ex(int dtype, int grad_dtype, int G, int P, int R, int ntiles,
                                  const int* tiles, const int* row_first, int heads, const void* qkv,
                                  int ldqkv, const void* ofwd, int ldof, const void* dout, int lddo,
                                  const float* lse, void* dqkv, int lddqkv, void* ws, size_t ws_bytes,
                                  int flags, void* stream);

/* Patch extraction: img fp32 [B,3,R,R] -> out [B*G*G, Kp] (out_dtype), K index c*p*p+ky*p+kx,
 * zero padded to Kp >= 3*p*p. */
int clipk_im2col(int out_dtype, int B, int res, int patch, int Kp, const float* img, void* out,
                 void* stream);

/* x[b*L + t] = ln_pre( (t==0 ? cls : patch[b*(L-1) + t-1]) + pos[t] ), L = G*G+1, f32 out. */
int clipk_vit_embed_ln(int B, int L, int width, const float* patch, const float* cls,
                       const float* pos, const float* gamma, const float* beta, float* x,
                       void* stream);

/* Prompt assembly (+ positional embedding) for nseq = B*C sequences of length L:
 *   s = b*C + c;  m = src_map[c*L + t]
 *   x0[s*L+t] = (m >= 0 ? emb[(c*77 + m)*W] : ctx[b*ctx_sb + c*ctx_sc + (-1-m)*W] + bias[b*W]) + pos[t*W]
 * bias may be NULL (CoOp). */
int clipk_prompt_assemble(int B, int C, int L, int W, const int* src_map, const float* emb,
                          const float* ctx, long ctx_sb, long ctx_sc, const float* bias,
                          const float* pos, float* x0, void* stream);

/* d ctx_shifted: dctx[b*out_sb + c*out_sc + k*W + w] = sum over c' in class group of
 *   dx0[((b*C + c')*L + pos_of(c',k))*W + w]   where pos_of from ctx_pos[c'*n_ctx + k].
 * csc != 0: one output per class (no sum over c). Deterministic fixed-order sums. */
int clipk_ctx_grad(int B, int C, int L, int W, int n_ctx, int csc, const int* ctx_pos,
                   const float* dx0, float* dctx, void* stream);

/* Packed-prompt assembly: x0[g*R + r] = token(c,t) (+ctx slot + bias[g]) + pos[t] with
 * c*L + t = row_tab[r] and the src_map convention above (ctx offset g*ctx_sg + c*ctx_sc). */
int clipk_prompt_assemble_rows(int G, int R, int C, int L, int W, const int* row_tab,
                               const int* src_map, const float* emb, const float* ctx, long ctx_sg,
                               long ctx_sc, const float* bias, const float* pos, float* x0,
                               void* stream);
/* dctx[(g*n_ctx + k)*W + w] = sum_{i in [slot_ptr[k], slot_ptr[k+1])} dx0[(g*R + slot_rows[i])*W + w]. */
int clipk_ctx_grad_rows(int G, int R, int W, int n_ctx, const int* slot_ptr, const int* slot_rows,
                        const float* dx0, float* dctx, void* stream);

/* CoCoOp's two prompt-parameter gradients of packed prompts in one launch (PromptAssembleFn
 * backward, cocoop.py:189-197 ctx_shifted = ctx + bias): with d(g, k) = the clipk_ctx_grad_rows
 * sum of slot k's rows of group g, dctx[k*W + w] = sum_g d(g, k)[w] (g order) and, when dbias is
 * given, dbias[g*W + w] = sum_k d(g, k)[w] (k order). Replaces the per-(g, k) output + two sums. */
int clipk_ctx_bias_grad_rows(int G, int R, int W, int n_ctx, const int* slot_ptr, const int* slot_rows,
                             const float* dx0, float* dctx, float* dbias, void* stream);

/* logits[b,c] = scale * <imf[b], txt[row]> / |txt[row]| / |imf[b]|,
 * row = per_image ? b*C + c : c.  tnorm[row] (optional out) = |txt[row]|. */
int clipk_cosine_logits_fwd(int B, int C, int E, int per_image, float scale, const float* imf,
                            const float* txt, float* logits, float* inv_tnorm, float* inv_inorm,
                            void* stream);
/* d txt[row] from dlogits (image side has no grad: frozen encoder). */
int clipk_cosine_logits_bwd(int B, int C, int E, int per_image, float scale, const float* imf,
                            const float* txt, const float* inv_tnorm, const float* inv_inorm,
                            const float* dlogits, float* dtxt, void* stream);

/* Row-wise CE / focal (gamma) loss with optional per-class alpha; writes per-row loss and
 * dlogits = d(mean loss)/dlogits * grad_scale. */
int clipk_ce_loss(int B, int C, const float* logits, const int64_t* labels, const float* alpha,
                  float gamma, int focal, float grad_scale, float* row_loss, float* dlogits,
                  void* stream);

/* clipk_ce_loss with the batch reduction in the same launch (one block): reduction 1 = mean,
 * 2 = sum of the row losses (summed in row order), into loss[0]; row_loss [B] is still written.
 * Replaces the separate mean / sum launch after clipk_ce_loss (coop.py:158-163 reductions). */
int clipk_ce_loss_reduce(int B, int C, const float* logits, const int64_t* labels, const float* alpha,
                         float gamma, int focal, float grad_scale, int reduction, float* row_loss,
                         float* loss, float* dlogits, void* stream);

/* CoCoOp Meta-Net: h = relu(x W1^T + b1); y = h W2^T + b2. x [B,V], W1 [Hd,V], W2 [Wd,Hd].
 * The CLIP widths (V % 256 == 0, V <= 1024, Hd <= 64, x / W1 16-B aligned) take the
 * many-block form; other shapes one block per image. */
int clipk_meta_net_fwd(int B, int V, int Hd, int Wd, const float* x, const float* w1,
                       const float* b1, const float* w2, const float* b2, float* h, float* y,
                       void* stream);
/* clipk_meta_net_fwd on the L2-normalised rows of x: xn [B,V] = x / |x| (written; cocoop.py:238
 * imf / imf.norm(dim=-1)), then the Meta-Net on xn -- the normalisation's two launches folded in. */
int clipk_meta_net_fwd_norm(int B, int V, int Hd, int Wd, const float* x, const float* w1,
                            const float* b1, const float* w2, const float* b2, float* xn, float* h,
                            float* y, void* stream);
/* grads of W1,b1,W2,b2 from dy (x has no grad). dh_ws: caller scratch of B*Hd floats. */
int clipk_meta_net_bwd(int B, int V, int Hd, int Wd, const float* x, const float* h,
                       const float* w2, const float* dy, float* dw1, float* db1, float* dw2,
                       float* db2, float* dh_ws, void* stream);

/* p -= lr * (buf = momentum*buf + (g + wd*p)); first step (has_buf==0): buf = g + wd*p. */
int clipk_sgd_step(long n, float* p, const float* g, float* buf, float lr, float momentum,
                   float weight_decay, int has_buf, void* stream);
/* clipk_sgd_step over up to 16 tensors of one param group in one launch (p[k], g[k], buf[k] of
 * n[k] floats, has_buf[k] per tensor; host arrays): the same per-element update. */
int clipk_sgd_step_multi(int count, float* const* p, const float* const* g, float* const* buf,
                         const long* n, const int* has_buf, float lr, float momentum,
                         float weight_decay, void* stream);

/* clipk_sgd_step_multi on grad_scale * g (e.g. 1 / world after a SUM all-reduce: the average
 * folded into the update instead of a division launch; 1.0 is bitwise clipk_sgd_step_multi). */
int clipk_sgd_step_multi_scaled(int count, float* const* p, const float* const* g, float* const* buf,
                                const long* n, const int* has_buf, float lr, float momentum,
                                float weight_decay, float grad_scale, void* stream);
/* clipk_sgd_step_multi_scaled skipped entirely (p, buf untouched) when guard[0] & mask != 0, read on
 * the device: the PREC fp32s trainer queues the step without waiting for its backward's overflow
 * flag (clipk_encoder_set_status bit 2) and re-runs an overflowed step later. */
int clipk_sgd_step_multi_if(int count, float* const* p, const float* const* g, float* const* buf,
                            const long* n, const int* has_buf, float lr, float momentum,
                            float weight_decay, float grad_scale, const int* guard, int mask, void* stream);
/* Status word hand-off (PREC fp32s overflow flags, clipk_encoder_set_status): host_word[0] =
 * flags[0], then flags[0] = 0, in one stream-ordered launch; host_word is host-visible memory
 * (pinned). The caller synchronises the stream (or an event after it) before reading it. */
int clipk_status_take(int* flags, int* host_word, void* stream);

/* Row gather / scatter: dst row (dst_rows ? dst_rows[i] : i) = src row (src_rows ? src_rows[i] : i)
 * for i < n; rows of row_bytes (multiple of 16) bytes, 16-B aligned. The text encoder's last
 * layer runs on the EOT rows only (the output is read there alone; exact) and moves rows
 * between the compact and the full layouts with it. */
int clipk_rows_copy(int row_bytes, int n, const void* src, const int* src_rows, void* dst,
                    const int* dst_rows, void* stream);

/* Elementwise cast fp32 -> dtype. */
int clipk_cast(int out_dtype, long n, const float* x, void* y, void* stream);

/* ---------------------------------------------------------------- encoders */
typedef struct clipk_encoder clipk_encoder;

/* Per-layer weight table order (n_per_layer = 16):
 *   0 ln1_w f32, 1 ln1_b f32, 2 in_w [3W,W] act, 3 in_b f32[3W], 4 out_w [W,W] act, 5 out_b,
 *   6 ln2_w, 7 ln2_b, 8 fc_w [4W,W] act, 9 fc_b f32[4W], 10 proj_w [W,4W] act, 11 proj_b,
 *   12 in_wT [W,3W] grad, 13 out_wT [W,W] grad, 14 fc_wT [W,4W] grad, 15 proj_wT [4W,W] grad
 * (12..15 may be NULL for a forward-only encoder). Head: lnf_w, lnf_b (f32), projT [E,W] act,
 * proj_grad [W,E] grad (NULL if forward-only).
 * act_dtype: forward GEMM operand type; grad_dtype: backward GEMM operand type. */
int clipk_encoder_create(int width, int layers, int heads, int embed, int act_dtype,
                         int grad_dtype, const void* const* layer_ptrs, const void* const* head_ptrs,
                         clipk_encoder** out);
void clipk_encoder_destroy(clipk_encoder* enc);

/* Deep prompts of an encoder (IVLP / MaPLe / PromptSRC, model.py:191-331): before layer l in
 * 1..n_deep the rows `rows` ([n_ctx][n_per], see clipk_rows_inject) of the residual stream
 * are replaced by prompts[l-1] ([n_deep][n_ctx][width] fp32, values as given: the trainers
 * round them through fp16 as the reference's .half() does); the backward writes the prompts'
 * gradients into grads[l-1] (when grads != NULL) and stops them there. Text: rows 1..n_ctx of
 * every sequence (packed layout: of every group); ViT: the last n_vpt rows of every image.
 * The pointers must stay valid for the calls that follow; n_deep = 0 clears. */
int clipk_encoder_set_deep_prompts(clipk_encoder* e, int n_deep, int n_ctx, int n_per, const int* rows,
                                   const float* prompts, float* grads);

/* Input-row mode of the next text-encoder calls on the shared-prefix packed layout
 * (clipk_text_{forward,backward}_packed). mode 0: every row of x0 is an independent input (the
 * reference's TextEncoder contract, coop.py:195-205). mode 1: only the P prefix rows of each
 * group carry per-group values -- the context slots of CoOp / CoCoOp with class position "end"
 * (coop.py:259-270; cocoop.py:173-198, pi_b added to ctx only) -- so the class rows of x0 are
 * identical in every group: layer 0's LN1 and qkv projection run once for them (group 0) and
 * are copied to the other groups, and the backward forms dx0 on the prefix rows only (the
 * rows clipk_ctx_grad_rows reads; the class rows of dx0 are left unspecified). Exact. Forward
 * and backward of one call must use the same mode. */
int clipk_encoder_set_input_rows(clipk_encoder* e, int mode);

/* LayerNorm fold of a 16-bit text encoder (see clipk_gemm_ln): fold_ptrs = 6 per layer,
 * {W_in' [3W, W] act dtype, s_in [3W] fp32, c_in [3W] fp32, W_fc' [4W, W], s_fc [4W], c_fc [4W]}
 * built from the layer's ln_1 / ln_2 and in_proj / c_fc weights. When set, layers >= 1 take
 * ln_1 from the previous layer's c_proj epilogue statistics and every layer takes ln_2 from its
 * out_proj epilogue (layer 0's ln_1 and ln_final stay LayerNorm passes; not used with deep
 * prompts or an fp32 encoder; a PREC fp32s encoder (clipk_encoder_set_split first) takes W_in' /
 * W_fc' split-packed). The saved mean / rstd are the same quantities the LayerNorm pass
 * writes, so the backward is unchanged. fold_ptrs == NULL clears. Pointers must stay valid. A ViT
 * handle (clipk_vision_create) takes the same table for its ln_1 / ln_2: its forward with a
 * 16-bit act dtype (clipk_vit_forward) runs the residual stream in that dtype through the text
 * encoder's layer loop and folds them the same way. */
int clipk_encoder_set_ln_fold(clipk_encoder* e, const void* const* fold_ptrs);

/* PREC fp32s on an fp32 encoder (act and grad dtype CLIPK_F32): on = 1 declares every GEMM weight
 * of the handle's tables (layer weights 2, 4, 8, 10 and their transposes 12-15; text head 2-3,
 * ViT head 4-5 and the prompted backward's proj) packed by clipk_split_pack, and runs every GEMM
 * of its calls as CLIPK_F32S (the fp32-class split-fp16 MFMA product). LayerNorm, attention and
 * the residual stream stay fp32. The text backward then runs on s * dtxt with s a power of two
 * from max |dtxt| (exact, undone on dx0 and the deep-prompt gradients), so the gradient operands
 * sit in fp16's normal range. Reference semantics: PromptSRC/clip/model.py:699 (fp32 model).
 * on = 2: those weights are fp16-valued (clipk_split_lo_zero returned 1 for each; the released
 * CLIP checkpoints) and the tables hold their COMPACT form (clipk_split_hi16) instead of the packed
 * one: every GEMM runs CLIPK_F32S16, 2 MFMAs per product, the same results as mode 1.
 * With a LayerNorm fold (clipk_encoder_set_ln_fold after this call) the fold tables then hold W
 * itself (compact) instead of W' = W diag(gamma), s = rowsums of W diag(gamma) over the packed
 * values / 64, and the fold GEMMs apply the layer's LayerNorm weight to A (clipk_gemm_ln_gamma).
 * The mode describes the tables' format, so it is fixed once set: a second call with another mode,
 * or any call after clipk_encoder_set_ln_fold, returns CLIPK_EINVAL. */
int clipk_encoder_set_split(clipk_encoder* e, int on);
/* The split backward's scale target t (default 7): s puts max |s dtxt| in [2^(t-1), 2^t). A lower
 * target leaves more headroom below fp16's 65504 for gradient growth through the layers, at
 * fewer significant bits for the smallest gradients. -24 <= t <= 30 (t > 16 overflows by design:
 * a test of the overflow status). */
int clipk_encoder_set_split_target(clipk_encoder* e, int target);
/* Overflow status of a PREC fp32s (split) encoder's calls: status = a device int the encoder
 * ORs flags into -- 1 when a text / ViT forward produced a non-finite feature, 2 when a backward's
 * returned gradients (dx0, deep-prompt and visual-prompt gradients) hold a non-finite value (the
 * split operands' fp16 range was exceeded: an activation or gradient past 65504). The caller zeroes
 * it and reads it when it synchronises (fsp_amd/clip/model.py re-runs an overflowed backward at a
 * lower scale target). NULL detaches. The pointer must stay valid for the calls that follow. */
int clipk_encoder_set_status(clipk_encoder* e, int* status);

/* ViT with visual prompts, forward with saved activations and input-grad backward (the
 * prompted VisionTransformer of IVLP / PromptSRC, model.py:401-431, and MaPLe, 434-485):
 * n_vpt prompt rows (vpt [n_vpt, width] fp32) appended after the image tokens before ln_pre,
 * deep prompts per clipk_encoder_set_deep_prompts, feat [B, E] fp32 from ln_post(CLS) @ proj.
 * saved == NULL: inference. The backward needs the encoder created with its transposed
 * layer weights (layer_ptrs 12..15) and proj_bwd = proj [width, E] in the grad dtype; it
 * writes d vpt [n_vpt, width] fp32 (summed over the images) and the deep prompts' gradients.
 * One workspace (clipk_vit_prompted_ws_bytes) serves both calls. */
size_t clipk_vit_prompted_saved_bytes(const clipk_encoder* e, int B, int n_vpt);
size_t clipk_vit_prompted_ws_bytes(const clipk_encoder* e, int B, int n_vpt);
int clipk_vit_forward_prompted(const clipk_encoder* e, int B, const float* img, int n_vpt, const float* vpt,
                               float* feat, void* saved, size_t saved_bytes, void* ws, size_t ws_bytes,
                               void* stream);
int clipk_vit_backward_prompted(const clipk_encoder* e, int B, int n_vpt, const float* vpt, const void* proj_bwd,
                                const float* dfeat, const void* saved, size_t saved_bytes, float* dvpt, void* ws,
                                size_t ws_bytes, void* stream);

/* Text encoder forward over nseq sequences of length L (x0 fp32 [nseq*L, W], positional
 * embedding already added). eot_rows[s] = s*L + EOT position of sequence s (int32, device).
 * txt fp32 [nseq, E].
 * If save != 0 the activations needed by clipk_text_backward stay in `saved`. */
size_t clipk_text_saved_bytes(const clipk_encoder* enc, int nseq, int L);
size_t clipk_text_ws_bytes(const clipk_encoder* enc, int nseq, int L);
int clipk_text_forward(const clipk_encoder* enc, int nseq, int L, const float* x0, const int* eot_rows,
                       float* txt, void* saved, size_t saved_bytes, void* ws, size_t ws_bytes,
                       void* stream);
size_t clipk_text_bwd_ws_bytes(const clipk_encoder* enc, int nseq, int L);
int clipk_text_backward(const clipk_encoder* enc, int nseq, int L, const int* eot_rows,
                        const float* dtxt, const void* saved, size_t saved_bytes, float* dx0,
                        void* ws, size_t ws_bytes, void* stream);

/* Shared-prefix packed variant (see clipk_attention_prefix_fwd): G groups of R rows,
 * C sequences per group, x0 fp32 [G*R, W]; eot_rows[g*C + c] = absolute EOT row;
 * txt fp32 [G*C, E]. Exact: rows after a sequence's EOT and duplicated causal prefixes
 * never influence the EOT features. */
size_t clipk_text_packed_saved_bytes(const clipk_encoder* enc, int G, int C, int R);
size_t clipk_text_packed_ws_bytes(const clipk_encoder* enc, int G, int C, int R);
size_t clipk_text_packed_bwd_ws_bytes(const clipk_encoder* enc, int G, int C, int R, int ntiles);
int clipk_text_forward_packed(const clipk_encoder* enc, int G, int C, int P, int R, int ntiles,
                              const int* tiles, const int* row_first, const float* x0,
                              const int* eot_rows, float* txt, void* saved, size_t saved_bytes,
                              void* ws, size_t ws_bytes, void* stream);
int clipk_text_backward_packed(const clipk_encoder* enc, int G, int C, int P, int R, int ntiles,
                               const int* tiles, const int* row_first, const int* eot_rows,
                               const float* dtxt, const void* saved, size_t saved_bytes, float* dx0,
                               void* ws, size_t ws_bytes, void* stream);

/* Vision transformer forward (frozen, no grad): img fp32 [B,3,R,R] -> feat fp32 [B,E]. With a
 * 16-bit act dtype the residual stream is kept in that dtype (CLIP's half semantics, as the text
 * encoder's; env CLIPK_VIT_RES16=0: fp32), ln_1 / ln_2 are folded when set
 * (clipk_encoder_set_ln_fold) and the last layer's post-attention half runs on the CLS rows.
 * Head table for a vision encoder: ln_pre_w, ln_pre_b, ln_post_w, ln_post_b (f32),
 * projT [E,D] act, conv_w [D,Kp] act, class_emb f32[D], pos f32[L,D]. */
int clipk_vision_create(int width, int layers, int heads, int embed, int res, int patch,
                        int act_dtype, const void* const* layer_ptrs,
                        const void* const* head_ptrs, clipk_encoder** out);
size_t clipk_vit_ws_bytes(const clipk_encoder* enc, int B);
int clipk_vit_forward(const clipk_encoder* enc, int B, const float* img, float* feat, void* ws,
                      size_t ws_bytes, void* stream);

/* Per-kernel-class timing with hipEvents on the launch stream (bench.py roofline). */
enum { CLIPK_PROF_NONE = 0, CLIPK_PROF_GEMM_FC = 1, CLIPK_PROF_GEMM_ALL = 2, CLIPK_PROF_ATTN = 3,
       CLIPK_PROF_LN = 4, CLIPK_PROF_GEMM_DGELU = 5 };
/* GEMM_FC = text c_fc forward GEMMs; GEMM_DGELU = text c_proj input-grad GEMMs with the fused
 * QuickGELU' epilogue; GEMM_ALL = every text GEMM; ATTN = text attention fwd+bwd. */
int clipk_prof_enable(int kind);
int clipk_prof_read(double* total_ms, long* count, double* flops_or_bytes);

/* Per-launch-site timing (bench.py's per-kernel roofline table): when on, every named launch
 * site of the encoders ("text.qkv_fwd", "text.attn_bwd", "text.ln_fwd", "vit.fc_fwd", ...) is
 * bracketed by hipEvents on its launch stream, with its algorithmic FLOPs and HBM bytes.
 * clipk_prof_sites_read fills up to max_sites rows (names: CLIPK_PROF_NAME_LEN chars each,
 * NUL-terminated) summed since the last read / enable, sets *n_sites, and resets. */
enum { CLIPK_PROF_NAME_LEN = 32 };
int clipk_prof_sites_enable(int on);
int clipk_prof_sites_read(int max_sites, char* names, double* total_ms, long* count, double* flops,
                          double* bytes, int* n_sites);

#ifdef __cplusplus
}
#endif
#endif /* CLIPK_H */
