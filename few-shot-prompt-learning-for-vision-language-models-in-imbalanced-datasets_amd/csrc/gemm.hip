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
#include <type_traits>

#include "common.h"

namespace clipk {

// residual / aux lookahead ring of the 256-row tiles, VGPRs: 16 = two row groups of a 16-bit
// aux (the dgelu GEMM's h) in flight; still no spill at 251 VGPRs. Same-box A/B
// (profiles/r02r/ab_xbud256.txt): dgelu 1.587 -> 1.488 ms/step, headline 11.92 -> 11.80 ms.
#ifndef CLIPK_XBUD256
#define CLIPK_XBUD256 16
#endif
#ifndef CLIPK_XBUD192
#define CLIPK_XBUD192 32
#endif
constexpr int GEMM_ROWB = 128;  // bytes per staged row (BK = 64 halfs / 32 floats)
constexpr int GEMM_NMIN = 128;  // N granularity accepted by the C-ABI
constexpr int EPI_SCRATCH = 16 * 64 * 4;  // per-wave epilogue transpose tile [16][64] fp32

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct GemmArgs {
  const char* A; const char* B;
  int M, N, K, lda, ldb;            // lda/ldb in elements
  const float* bias; const void* res; int ldr;  // res: TX (fp32, or the 16-bit out dtype)
  void* out; int ldo; void* out2;
  const void* aux; int ldaux;
  unsigned long long* stamp;  // diagnostic (CLIPK_GEMM_STAMP): per block/tile s_memrealtime marks
  int ksplit;                 // split-K slices (non-persistent only); slice s writes out + s*split_stride
  long long split_stride;     // elements of TO between slices' fp32 partial outputs
  int skew;                   // persistent kernels: ~us of start delay for every other CU of an XCD
  // LayerNorm folded into the GEMMs (clipk_gemm_ln): LNM 1 writes per (row, 64-column group)
  // statistics partials of the rounded output to lnstats; LNM 2 applies LN to A = x through the
  // epilogue rstd * acc - rstd * mean * colsum + bias (B = W diag(gamma), bias = b + W beta) with
  // the rows' (rstd, -rstd * mean) pairs (clipk_ln_stats_merge of the producer's partials)
  float* lnstats;
  const float* colsum;
  const f32x2* lnrnb;
  // LNM 3 (clipk_gemm_ln_merge): the fold reads the producer's partials (lnstats) and merges each
  // row's itself, exactly as clipk_ln_stats_merge; the column-0 tiles write mean / rstd / rnb
  float* lnmean; float* lnrstd; f32x2* lnrnb_out;
  // LNM 4 (clipk_gemm_ln_gamma, PREC fp32s): LNM 2 with B = W itself and the LayerNorm weight
  // applied to A instead, x[m, k] * gamma[k] in fp32 before the split (K <= kGammaMax); colsum =
  // rowsums of W diag(gamma). Keeps W fp16-valued, so the fold runs CLIPK_F32S16's 2 MFMAs
  const float* lngamma;
};
constexpr int kGammaMax = 1024;

// Sum over the aligned 8-lane group (DPP: quad xor 1, quad xor 2, half-row mirror i <-> 7 - i).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float sum8(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  return v + dpp_f<0x141>(v);
}
// Sum over the aligned 8- or 16-lane group (16: + the row mirror i <-> 15 - i, the other half)
template <int L>
__device__ __forceinline__ float sum_group(float v) {
  v = sum8(v);
  if constexpr (L == 16) v += dpp_f<0x140>(v);
  return v;
}
constexpr int STAMP_TILES = 8, STAMP_BLOCKS = 2048;

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

// ---- PREC fp32s (CLIPK_F32S): fp32-class products on the 16-bit MFMA.
// 8 fp32 values (a lane's two 16-B fragment chunks, k = 8 fq .. 8 fq + 7) -> fp16 hi = fp16(x)
// and lo = fp16(x - hi): hi + lo carries ~22 significant bits of x.
// The lo part is one mixed-precision FMA per element: fp16(a * 1 - f32(h)) reads h straight
// from the packed fp16 register and rounds once (exact: x - hi is representable in fp32), so
// a pair costs 1 cvt_pk + 2 fma_mix instead of cvt_pk + 2 cvt + sub + cvt_pk (the split sits in
// the ping-pong loop's memory segment, where its VALU count is on the critical path).
#ifndef CLIPK_SPLIT_MIX
#define CLIPK_SPLIT_MIX 1
#endif
__device__ __forceinline__ unsigned split_lo2(float a, float b, unsigned h) {
  unsigned l;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(l)
      : "v"(a), "v"(b), "v"(h));
  return l;
}
// MIX false: the lo part in compiler-visible cvt + sub + cvt form. The v_fma_mix pair is inline
// asm, whose VGPR writes the compiler's hazard tracking does not see: an MFMA that reads them a
// few instructions later (the 2- / 4-slot loop, where splits and MFMAs interleave) can read
// stale values -- measured: the 2-MFMA split kernel on the 128x128 tiles off by up to 5e-2 at
// 4k-8k rows, bit-exact with this form or with s_nop 7 after the split
// (profiles/r05w16/hazard.txt). The ping-pong loop splits in its memory segment, a barrier
// before the MFMAs that read the parts, and keeps the cheaper asm form.
template <bool MIX = CLIPK_SPLIT_MIX != 0>
__device__ __forceinline__ void split8(u32x4 a0, u32x4 a1, u32x4& hi, u32x4& lo) {
  const f32x4 x0 = __builtin_bit_cast(f32x4, a0), x1 = __builtin_bit_cast(f32x4, a1);
  f16x8 h;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    h[c] = (f16)x0[c];
    h[4 + c] = (f16)x1[c];
  }
  hi = __builtin_bit_cast(u32x4, h);
  if constexpr (!MIX) {  // (also the A/B knob CLIPK_SPLIT_MIX=0 everywhere)
    f16x8 l;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      l[c] = (f16)(x0[c] - (float)h[c]);
      l[4 + c] = (f16)(x1[c] - (float)h[4 + c]);
    }
    lo = __builtin_bit_cast(u32x4, l);
    return;
  }
  lo[0] = split_lo2(x0[0], x0[1], hi[0]);
  lo[1] = split_lo2(x0[2], x0[3], hi[1]);
  lo[2] = split_lo2(x1[0], x1[1], hi[2]);
  lo[3] = split_lo2(x1[2], x1[3], hi[3]);
}
// a . b ~= hi(a) hi(b) + hi(a) lo(b) + lo(a) hi(b) (lo . lo ~ 2^-22 relative is dropped); the
// weight's parts (packed, clipk_split_pack) are the instruction's A operand (swapped operands)
// Precision experiment (build-time, A/B only): CLIPK_SPLIT_TERMS 2 drops the
// lo(a) hi(b) term -- the activation operand rounded to fp16, the weight kept at ~22 bits -- in
// the GEMMs of epilogue class `CLIPK_SPLIT_TERMS_EPI` (0: every GEMM, 1: the backward's input-grad
// GEMMs, EPI_NONE / EPI_DMUL / EPI_DQGELU).
#ifndef CLIPK_PP_SPLIT_NOP  // 0: none; n > 0: s_nop (n - 1) after the ping-pong loop's split (5: measured free, profiles/r05w16/ppnop_*.txt)
#define CLIPK_PP_SPLIT_NOP 5
#endif
#ifndef CLIPK_SPLIT_TERMS
#define CLIPK_SPLIT_TERMS 3
#endif
#ifndef CLIPK_SPLIT_TERMS_EPI
#define CLIPK_SPLIT_TERMS_EPI 0
#endif
// W16 (CLIPK_F32S16): lo(b) is zero, so the hi(a) lo(b) product adds exact zeros and is skipped
// (the compiler then drops the lo(b) fragment reads from LDS too)
template <bool TWO = false, bool W16 = false>
__device__ __forceinline__ f32x4 mma_split(u32x4 bh, u32x4 bl, u32x4 ah, u32x4 al, f32x4 c) {
  if constexpr (!W16)
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, bl), __builtin_bit_cast(f16x8, ah), c, 0, 0, 0);
  if constexpr (!TWO)
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, bh), __builtin_bit_cast(f16x8, al), c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, bh), __builtin_bit_cast(f16x8, ah), c, 0,
                                                0, 0);
}
constexpr float kSplitAlpha = 1.0f / CLIPK_SPLIT_SCALE;  // the packed weights' scale, undone

// Training's QuickGELU pair with the derivative saved (CLIPK_QGELU_DERIV, include/clipk.h):
// internal epilogue ids next to the public CLIPK_EPI_* ones
constexpr int EPI_QGELU_D = 5;  // out = quickgelu(acc + bias), out2 = quickgelu'(acc + bias)
constexpr int EPI_DMUL = 6;     // out = acc * aux (aux: the saved quickgelu')
constexpr bool epi_qgelu(int e) { return e == CLIPK_EPI_BIAS_QGELU || e == EPI_QGELU_D; }

__device__ __forceinline__ void glds16(const char* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(
      (const __attribute__((address_space(1))) void*)src,
      (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// Raw bytes of one lane's epilogue operand run (residual f32 / aux TX, CW columns), kept
// unconverted until use: a conversion right after the load would wait for it.
template <int NB> struct Raw;
template <> struct Raw<8> { uint2 v; };
template <> struct Raw<16> { uint4 v; };
template <> struct Raw<32> { uint4 v[2]; };

// Cache policy of the epilogue's streaming traffic (build-time A/B knobs, tools/ab_bench.sh):
// CLIPK_GEMM_SPOL = the output stores' cache-policy bits, CLIPK_GEMM_XNT = non-temporal
// residual / aux loads. Headline step (profiles/r02k_ab_cache_policy.txt): plain 12.70 ms;
// nt stores (2) 12.43 -- every GEMM 4-9 % faster, their consumers (LayerNorm, attention) a
// little slower; sc1 stores (16, the line leaves the XCD's L2) 12.72; nt stores + nt aux /
// residual loads 12.37-12.43 (dgelu 1.61 -> 1.55 ms/step): the default.
#ifndef CLIPK_GEMM_SPOL
#define CLIPK_GEMM_SPOL 2
#endif
#ifndef CLIPK_GEMM_XNT
#define CLIPK_GEMM_XNT 1
#endif
// Store policy of a residual stream written with LN statistics (clipk_gemm_ln producers): its
// consumer is the next GEMM's A operand, re-read by every column tile, so the lines are kept
// (plain stores) rather than streamed past the caches. Same-box A/B of the fold
// (profiles/r03c/ab_lnfold.txt): with nt stores the folded c_fc ran 0.24 ms/step slower than
// the LayerNorm-pass c_fc; with plain stores 0.04 ms.
#ifndef CLIPK_GEMM_SPOL_LN
#define CLIPK_GEMM_SPOL_LN 0
#endif
// Store policy of the outputs the NEXT GEMM reads as its A operand: c_fc's QuickGELU(h) (c_proj,
// forward) and dgelu's dh (fc_dx, backward). c_fc's second output (the saved QuickGELU', read a
// whole forward + backward later) keeps CLIPK_GEMM_SPOL.
#ifndef CLIPK_GEMM_SPOL_CHAIN
#define CLIPK_GEMM_SPOL_CHAIN 2
#endif
// CLIPK_GEMM_PP: 192x256 / 256x256 launches with >= 2 K tiles run the ping-pong main loop
// (1, persistent; 2 = one tile per block, A/B; 0 = the 2-slot loop). Same-box A/B
// (profiles/r02m_ab_pingpong.txt): headline step 12.60 -> 12.13 ms, input-grad GEMMs
// 2.65 -> 2.27 ms/step; staging by global_load_lds with per-lane 64-bit addresses instead of
// buffer LDS-DMA measured 12.80 ms (the address arithmetic sits in the memory segments).
#ifndef CLIPK_GEMM_PP
#define CLIPK_GEMM_PP 1
#endif
// CLIPK_GEMM_RING (A/B): 192x256 launches as non-persistent 4-slot rings of 64-B K steps.
#ifndef CLIPK_GEMM_RING
#define CLIPK_GEMM_RING 0
#endif
// CLIPK_GEMM_PPB0: the ping-pong loop keeps phase 1's B-half-0 fragments in registers for
// phase 4 instead of re-reading them (4 of 24 ds_read_b128 per wave and K tile, +13-16 VGPRs,
// no spill at 256 rows). Same-box A/B (profiles/r02o_ab_ppb0.txt): headline step 11.91 ->
// 11.82 ms, input-grad GEMMs 2.195 -> 2.166 ms/step.
#ifndef CLIPK_GEMM_PPB0
#define CLIPK_GEMM_PPB0 1
#endif
// CLIPK_GEMM_PP2: the ping-pong loop in 2 phases per K tile instead of 4 -- (A half 0 x all of
// B), (A half 1 x all of B), B's fragments read once and kept in registers -- so each wave
// crosses 4 barriers per K tile instead of 8 and each MFMA segment is 24 MFMAs instead of 12.
// Restage: A1 + B1 of K tile t+1 in phase 1, A0 + B0 of t+2 in phase 2 (each one phase after
// its last read by the lagging wave row); phase 2's counted vmcnt leaves only those in flight.
// 1 = every ping-pong tile, 2 = the 256-row tiles only (default), 0 = off. Same-box A/Bs
// (profiles/r03i/ab_pp2.txt): on the 256-row tiles (qkv / c_fc forward, dgelu) 1-3 % faster per
// launch, headline 10.70 -> 10.57 ms/step; on the 192-row tiles (the N = 512 GEMMs) 1-2 % slower.
// PMC over both shapes: no LDS bank conflicts or unaligned replays, the LDS array busy ~25 % and
// the MFMA pipes ~45 % of the kernel's cycles -- the loop is bound by its issue / synchronisation
// structure rather than by either unit.
#ifndef CLIPK_GEMM_PP2
#define CLIPK_GEMM_PP2 2
#endif
// CLIPK_GEMM_PRIO (A/B): wave priority in the ping-pong loop -- 1 = the MFMA segment runs at
// priority 1 (default), 0 = no priority changes, 2 = the memory segment (fragment reads,
// restage issue) runs at priority 1 instead.
#ifndef CLIPK_GEMM_PRIO
#define CLIPK_GEMM_PRIO 1
#endif
// CLIPK_GEMM_APOL (A/B, build-time): cache-policy bits of the ping-pong loop's A-operand LDS-DMA
// (0 default; the staging lab read 100 -> 96.5 us with sc0 (1) or sc1 (16), profiles/r05zh/)
#ifndef CLIPK_GEMM_APOL
#define CLIPK_GEMM_APOL 0
#endif
// CLIPK_GEMM_WARM (A/B, build-time; 0 = off): the 192-row ping-pong loop (16-bit) touches one
// dword of every 128-B line of the A panel CLIPK_GEMM_WARM K steps ahead (waves 0-2, one line per
// lane), so the first read of each activation line is in flight before its LDS-DMA. The staging
// lab measured 100 -> 94 us for this tile's operand stream at 2 steps ahead
// (tools/lab/stage_lab.hip, profiles/r05zh/).
#ifndef CLIPK_GEMM_WARM
#define CLIPK_GEMM_WARM 0
#endif
// Diagnostic builds only (wrong results; tools/gemm_diag.sh): NOLOAD = stage no K step past
// the first (the loop's compute + LDS + barrier ceiling), NOBAR = no barrier / vmcnt wait per
// K step either.
#ifndef CLIPK_GEMM_NOLOAD
#define CLIPK_GEMM_NOLOAD 0
#endif
#ifndef CLIPK_GEMM_NOBAR
#define CLIPK_GEMM_NOBAR 0
#endif
// NOMMA = no MFMA in the ping-pong loop (its load + LDS + barrier time alone).
#ifndef CLIPK_GEMM_NOMMA
#define CLIPK_GEMM_NOMMA 0
#endif
template <int NB> __device__ __forceinline__ void ld_raw(const void* p, Raw<NB>& r) {
#if CLIPK_GEMM_XNT
  typedef unsigned int nt2 __attribute__((ext_vector_type(2)));
  typedef unsigned int nt4 __attribute__((ext_vector_type(4)));
  if constexpr (NB == 8) {
    r.v = __builtin_bit_cast(uint2, __builtin_nontemporal_load(reinterpret_cast<const nt2*>(p)));
  } else if constexpr (NB == 16) {
    r.v = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const nt4*>(p)));
  } else {
    r.v[0] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const nt4*>(p)));
    r.v[1] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const nt4*>(p) + 1));
  }
#else
  if constexpr (NB == 8) r.v = *reinterpret_cast<const uint2*>(p);
  else if constexpr (NB == 16) r.v = *reinterpret_cast<const uint4*>(p);
  else { r.v[0] = reinterpret_cast<const uint4*>(p)[0]; r.v[1] = reinterpret_cast<const uint4*>(p)[1]; }
#endif
}
template <typename TX, int CW, int NB>
__device__ __forceinline__ void raw_f32(const Raw<NB>& r, float* o) {
  static_assert(CW * (int)sizeof(TX) == NB, "raw run size");
  const TX* e = reinterpret_cast<const TX*>(&r);
#pragma unroll
  for (int c = 0; c < CW; ++c) o[c] = to_f32(e[c]);
}
// CW (4 or 8) consecutive fp32 values -> TO in memory (one 8/16-B store).
template <typename TO, int CW>
__device__ __forceinline__ void store_run(TO* p, const float* v) {
  if constexpr (CW == 8) store16_f32<TO>(p, v);
  else store4<TO>(p, v[0], v[1], v[2], v[3]);
}

// Epilogue stores go through a buffer resource spanning the tile's valid rows: a lane whose
// row is past M stores out of range and the hardware drops it, so no lane branches around
// its store. (A branch there made the compiler's vmcnt bookkeeping merge a stored / not
// stored path at every row group and wait vmcnt(0) -- for every earlier store -- in each.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void* base, long long bytes) {
  const unsigned n = bytes <= 0 ? 0u : bytes >= 0x7fffffffLL ? 0x7fffffffu : (unsigned)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)n, 0x00020000);
}
// 16 bytes of TO (16 / sizeof(TO) fp32 values converted) at byte offset off
template <typename TO, int POL = CLIPK_GEMM_SPOL>
__device__ __forceinline__ void buf_store16(__amdgpu_buffer_rsrc_t r, int off, const float* v) {
  u32x4 d;
  if constexpr (sizeof(TO) == 4) {
    d = __builtin_bit_cast(u32x4, (f32x4){v[0], v[1], v[2], v[3]});
  } else {
    typedef TO t8 __attribute__((ext_vector_type(8)));
    t8 h;
#pragma unroll
    for (int c = 0; c < 8; ++c) h[c] = (TO)v[c];
    d = __builtin_bit_cast(u32x4, h);
  }
  __builtin_amdgcn_raw_buffer_store_b128(d, r, off, 0, POL);
}

// Start skew (knob CLIPK_GEMM_SKEW, ~us): every other CU of each XCD starts late, so that the
// persistent blocks' store-heavy epilogues stop landing on HBM all at once.
__device__ __forceinline__ void skew_start(int us, int bid) {
  if (us > 0 && ((bid >> 3) & 1))
    for (int i = 0; i < us; ++i) __builtin_amdgcn_s_sleep(32);  // 64 x 32 cycles each
}

// Raw barrier pinned in program order: glds may stay in flight across it (a __syncthreads()
// would make the compiler drain them with vmcnt(0)).
#define G8_BAR()                       \
  do {                                 \
    __builtin_amdgcn_sched_barrier(0); \
    __builtin_amdgcn_s_barrier();      \
    __builtin_amdgcn_sched_barrier(0); \
  } while (0)

// Block tile BM x BN, WM x WN waves (each (BM/WM) x (BN/WN) = TM x TN 16x16 sub-tiles),
// 2-stage LDS ring, one barrier per 128-byte K step. PERSIST: the grid is sized to the
// CU count and each block walks an XCD-contiguous run of tiles; the last K step of a tile
// prefetches the first stage of the next tile, so that load overlaps the epilogue.
// DEPTH > 2 (non-persistent only): a DEPTH-slot LDS ring with DEPTH-1 stages in flight, a
// counted vmcnt and a raw barrier per K step -- for the latency-bound small-M GEMMs (the ViT's
// 1,576-row projections: one tile per CU, where a 2-slot ring waits out a load latency every
// 64-deep K step).
// AG (CLIPK_A_QGELU, non-persistent 2-slot only): A is a pre-activation h; each thread loads
// its A chunks of the next stage into registers at the top of a K step (where the glds would
// have been issued), and after the step's MFMAs writes quickgelu(h) to the same lane-linear
// LDS slots the glds would have filled.
// PP (ping-pong, non-persistent 8-wave 2x4 tiles of BN = 256, 16-bit): each 64-deep K tile
// runs as 4 phases, one output quadrant each -- (A half 0, B half 0), (A0, B1), (A1, B1),
// (A1, B0), where A half h = rows h*BM/4.. of each wave row's BM/2 and B half q = columns
// q*32.. of each wave column's 64 -- and every phase is a memory segment (this phase's
// fragment reads + one region's glds restage, lgkmcnt(0)) and an MFMA segment, each ended by a
// raw barrier. Wave row 1 starts one barrier late, so on every SIMD one wave's MFMAs overlap
// the other's LDS reads. A region is restaged (for K tile t+2, or t+1 for B0) one phase after
// its last read; the K tile t+1 wait is a counted vmcnt at phase 4 of tile t that leaves the
// three regions already issued for t+2 in flight -- the ring never drains in the loop.
// LNM (clipk_gemm_ln): 1 = per-row LayerNorm statistics of the output, 2 = LayerNorm of A,
// 3 = LNM 2 with the statistics merge of clipk_ln_stats_merge inside (clipk_gemm_ln_merge)
// folded into the epilogue (see GemmArgs).
template <typename T, typename TO, typename TX, int EPI, int BM, int BN, int WM, int WN, bool PERSIST,
          int ROWB = GEMM_ROWB, int DEPTH = 2, bool AG = false, bool PP = false, int LNM = 0>
__global__ __launch_bounds__(WM * WN * 64, DEPTH == 2 ? 2 : 1) void gemm_nt_kernel(GemmArgs g) {
  static_assert(DEPTH == 2 || !PERSIST, "deep ring: non-persistent launches only");
  static_assert(!AG || (!PERSIST && DEPTH == 2 && sizeof(T) == 2 && ROWB == 128), "A-operand QuickGELU path");
  // PREC fp32s: 4-byte elements (A fp32, B split-packed), staged as fp32; a 128-B K step is
  // one 32-deep k-window read as two 16-B chunks per fragment (2 fq, 2 fq + 1), 3 MFMAs each
  constexpr bool SPLIT = is_split_v<T>, W16 = __is_same(T, f32h);
  constexpr bool LN_GAMMA = LNM == 4;
  static_assert(!LN_GAMMA || SPLIT, "gamma-on-A fold: split GEMMs");
  [[maybe_unused]] constexpr bool TWO_TERMS =
      CLIPK_SPLIT_TERMS == 2 && (CLIPK_SPLIT_TERMS_EPI == 0 || EPI == CLIPK_EPI_NONE || EPI == CLIPK_EPI_DQGELU ||
                                 EPI == EPI_DMUL);
  static_assert(!SPLIT || (ROWB == 128 && !AG), "split-fp16 GEMM: 128-B staged rows");
  static_assert(!PP || (PERSIST && !AG && DEPTH == 2 && ROWB == 128 && WM == 2 && WN == 4 && BN == 256 &&
                        (sizeof(T) == 2 || SPLIT) && BM % 64 == 0), "ping-pong main loop (K >= 128)");
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int OPA = BM * ROWB, OPB = BN * ROWB, STAGE = OPA + OPB;
  constexpr int RPI = 1024 / ROWB;   // rows per glds wave-instruction (64 lanes x 16 B)
  constexpr int CPR = ROWB / 16;     // 16-B chunks per staged row
  constexpr int KK = ROWB / 64;      // 64-B MFMA k-windows per K step
  // A stage is NG glds units of RPI rows (1 KiB each, A's GA units then B's), unit g landing
  // at stage offset g * 1024. BLOCKED (every wave the same number of A and of B units): wave w
  // issues A units w*IA.. and B units GA + w*IB..; otherwise units are dealt round-robin
  // (g = w + NW*i) and the first NREM waves issue one more than the others.
  constexpr int GA = BM / RPI, GB = BN / RPI, NG = GA + GB;
  constexpr bool BLOCKED = GA % NW == 0 && GB % NW == 0;
  constexpr int IA = BLOCKED ? GA / NW : 0, IB = BLOCKED ? GB / NW : 0;
  constexpr int NI = (NG + NW - 1) / NW;  // glds slots per wave (the last may be idle)
  constexpr int PERL = NG / NW, NREM = NG % NW;
  static_assert(ROWB == 128 || (ROWB == 64 && sizeof(T) == 2), "staged row is 128 B (or 64 B for 16-bit)");
  static_assert(BM % RPI == 0 && BN % RPI == 0 && NG >= NW, "tile/wave mismatch");
  static_assert(!AG || BLOCKED, "A-operand QuickGELU path: blocked unit split");
  // (+ 1 KiB: the CLIPK_GEMM_WARM junk area of the 192-row ping-pong loop)
  constexpr int WARM_B = CLIPK_GEMM_WARM > 0 && PP && BM == 192 ? 1024 : 0;
  constexpr int GAM_OFF = DEPTH * STAGE + NW * EPI_SCRATCH + WARM_B;  // LNM 4: gamma[K] in LDS
  __shared__ CLIPK_LDS_ALIGN char smem[GAM_OFF + (LN_GAMMA ? kGammaMax * 4 : 0)];  // one array (see header)
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // ---- XCD-aware bijective tile split: XCD group x owns tiles [t_beg, t_end) (row-panel
  // major, so the tiles sharing an A panel run on one XCD and re-read it from its L2).
  // Split-K (non-persistent only): units are slice-major, so neighbouring units are
  // neighbouring tiles over the same K range (shared panels in L2).
  const int ntn = g.N / BN;
  const int ntm = (g.M + BM - 1) / BM;
  const int ntiles = ntm * ntn;
  const int nwg = ntiles * (PERSIST ? 1 : g.ksplit);
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int t_beg = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int t_end = t_beg + (xcd < r ? q + 1 : q);
  const int t_step = PERSIST ? (int)(gridDim.x >> 3) : 1;
  int tile = t_beg + (bid >> 3);
  if (tile >= t_end) return;  // block-uniform
  if constexpr (PERSIST) skew_start(g.skew, bid);
  const int ks = PERSIST ? 0 : tile / ntiles;
  if (!PERSIST) tile -= ks * ntiles;

  const size_t esz = sizeof(T);
  const int nk_all = (int)((size_t)g.K * esz / ROWB);
  const int kt0 = PERSIST ? 0 : ks * nk_all / g.ksplit;
  const int nk = PERSIST ? nk_all : (ks + 1) * nk_all / g.ksplit - kt0;
  TO* const outb = (TO*)g.out + (PERSIST ? 0 : (size_t)ks * g.split_stride);
  // source-side swizzle of 16-B chunk c in row r: 128-B rows c ^ ((r >> 1) & 7), 64-B rows
  // c ^ ((r >> 2) & 3) -- either way 16 consecutive rows read at one chunk hit 16 distinct
  // 16-B slots of the 256-B bank row
  auto swz = [](int r) { return ROWB == 128 ? (r >> 1) & 7 : (r >> 2) & 3; };
  auto unit = [&](int i) { return BLOCKED ? (i < IA ? w * IA + i : GA + w * IB + (i - IA)) : w + NW * i; };
  const char* src[NI];
  auto set_tile = [&](int t) {
    const int tm0 = (t / ntn) * BM, tn0 = (t % ntn) * BN;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int u = unit(i);
      const bool ua = BLOCKED ? i < IA : u < GA;
      const int row = (ua ? u : u - GA) * RPI + lane / CPR;
      const int c = (lane % CPR) ^ swz(row);  // source-side swizzle
      if (ua) {
        int ga = tm0 + row;
        ga = ga < g.M ? ga : g.M - 1;
        src[i] = g.A + ((size_t)ga * g.lda) * esz + c * 16 + (size_t)kt0 * ROWB;
      } else {
        const int gb = u < NG ? tn0 + row : tn0;  // idle slot: a valid address, never issued
        src[i] = g.B + ((size_t)gb * g.ldb) * esz + c * 16 + (size_t)kt0 * ROWB;
      }
    }
  };
  u32x4 ra[AG ? IA : 1];  // AG: the next stage's A chunks in flight
  auto stage = [&](int s, int kt) {
    if (CLIPK_GEMM_NOLOAD && kt > 0) return;
    char* base = smem + s * STAGE;
    const size_t koff = (size_t)kt * ROWB;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if constexpr (AG) {
        if (i < IA) {
          ra[i] = *reinterpret_cast<const u32x4*>(src[i] + koff);
          continue;
        }
      }
      const int u = unit(i);
      if (BLOCKED || NREM == 0 || u < NG) glds16(src[i] + koff, base + u * 1024);
    }
  };
  auto write_a = [&](int s) {  // AG: quickgelu of the loaded chunks into stage s
    if constexpr (AG) {
      typedef T t8 __attribute__((ext_vector_type(8)));
      char* base = smem + s * STAGE;
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        t8 hv = __builtin_bit_cast(t8, ra[i]);
#pragma unroll
        for (int c = 0; c < 8; ++c) hv[c] = (T)quick_gelu((float)hv[c]);
        *reinterpret_cast<u32x4*>(base + (w * IA + i) * 1024 + lane * 16) = __builtin_bit_cast(u32x4, hv);
      }
    }
  };

  const int wm = w / WN, wn = w % WN;
  const int fr = lane & 15;         // fragment row within a 16-row sub-tile
  const int fq = lane >> 4;         // 16-B chunk within a 64-B k-window
  const int sw = swz(fr);           // row swizzle (sub-tile row base is a multiple of 16)
  constexpr bool HAS_BIAS = EPI == CLIPK_EPI_BIAS || EPI == CLIPK_EPI_BIAS_RES || epi_qgelu(EPI);
  constexpr bool HAS_EXT = EPI == CLIPK_EPI_BIAS_RES || EPI == CLIPK_EPI_DQGELU || EPI == EPI_DMUL;

  if constexpr (LN_GAMMA) {  // the LayerNorm weight, once per block (before any LDS-DMA is issued)
    for (int k = threadIdx.x; k < g.K; k += NW * 64) reinterpret_cast<float*>(smem + GAM_OFF)[k] = g.lngamma[k];
    __syncthreads();
  }
  [[maybe_unused]] const float* sgam = reinterpret_cast<const float*>(smem + GAM_OFF);
  set_tile(tile);
  // deep ring: wait until stage kt+1 has landed while `younger` later stages stay in flight
  // (this wave's glds per stage: PERL, or PERL + 1 for the first NREM waves)
  auto ring_wait = [&](int younger) {
    if constexpr (DEPTH > 2) {
      if (NREM != 0 && w < NREM) {
        constexpr int P = PERL + 1;
        if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * P) : "memory");
        else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        constexpr int P = PERL;
        if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * P) : "memory");
        else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
  };
  static_assert(DEPTH <= 4, "ring_wait covers up to two younger stages");
  if constexpr (PP) {
    // prologue inside the tile loop
  } else if constexpr (DEPTH == 2) {
    stage(0, 0);
    write_a(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
    for (int d = 0; d < DEPTH - 1; ++d)
      if (d < nk) stage(d, d);
    ring_wait(min(DEPTH - 2, nk - 1));
    G8_BAR();
  }
  int it = 0;  // global K-step counter (LDS buffer = it & 1)
  int ti = 0;  // tiles done by this block (diagnostic stamps)
  unsigned long long* stp = (g.stamp && threadIdx.x == 0 && bid < STAMP_BLOCKS)
                                ? g.stamp + (size_t)bid * (STAMP_TILES * 3 + 4) : nullptr;
  if (stp) { stp[0] = __builtin_amdgcn_s_memtime(); stp[1] = __builtin_amdgcn_s_memrealtime(); }

  const int kt0c = kt0, nkc = nk, kt0n = 0;  // this tile's K range, the next tile's first K step
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
    // read-back geometry: each lane owns CW consecutive columns of one row, so every store /
    // residual / aux instruction moves 16 B per lane (8 columns of a 16-bit output, 4 of fp32)
    // and covers RPQ rows x 64 columns
    constexpr int CW = sizeof(TO) == 2 ? 8 : 4;
    constexpr int LPR = 64 / CW, RPQ = 64 / LPR, NQ = 16 / RPQ;
    const int er = lane / LPR, ec = lane % LPR;
    const int ncol = nbase + CW * ec;
    // residual / aux operands run XD groups ahead of the group being stored (a register ring
    // of <= 32 VGPRs): aux h comes from HBM, and one group of lookahead left every group
    // waiting out a full load latency (dgelu epilogue 8.8 us per 256x256 tile)
    constexpr int XNB = CW * (int)sizeof(TX);
    typedef Raw<XNB> XR;
    constexpr int XREG = NQ * XNB / 4;
    // ring VGPRs (256-row tiles: little to spare; the LN-statistics epilogue needs 8 more)
    constexpr int XBUD = BM == 192 ? CLIPK_XBUD192 : (LNM == 1 ? CLIPK_XBUD256 / 2 : CLIPK_XBUD256);
    constexpr int XD = XBUD / XREG < 1 ? 1 : (XBUD / XREG > TM ? TM : XBUD / XREG);
    XR extq[XD][NQ];
    auto load_ext = [&](int i, XR* dst) {
      if constexpr (HAS_EXT) {
        const int mg = m0 + wm * (BM / WM) + i * 16;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          int mc = mg + RPQ * q + er;
          mc = mc < g.M ? mc : g.M - 1;
          if constexpr (EPI == CLIPK_EPI_BIAS_RES)
            ld_raw<XNB>((const TX*)g.res + (size_t)mc * g.ldr + ncol, dst[q]);
          else
            ld_raw<XNB>((const TX*)g.aux + (size_t)mc * g.ldaux + ncol, dst[q]);
        }
      }
    };
    // LN fold: mean / rstd of the lane's rows, two 16-row groups ahead of their use. (Merging the
    // producer's partials here instead of in clipk_ln_stats_merge -- 2 loads + 2 8-lane sums per
    // row -- measured slower: qkv 86 -> 110 us, c_fc 129 -> 158 us per launch.)
    constexpr bool LN_IN = LNM == 2 || LNM == 3 || LNM == 4, LN_OUT = LNM == 1, LN_MERGE = LNM == 3;
    // LN_MERGE: 16-bit out (8 lanes per row = the 8 partials of W = 512: lane ec merges partial
    // ec, the merge kernel's lane map and DPP order, so the same bits) on the 192-row ping-pong
    // tiles, whose free residual ring holds the tile's partials (loaded at the tile's start)
    static_assert(!LN_MERGE || (PP && BM == 192 && sizeof(TO) == 2), "in-kernel LN statistics merge");
    // (16-bit out: 8 lanes per row of 64 columns; PREC fp32s, fp32 out: 16)
    static_assert(!LN_OUT || (EPI == CLIPK_EPI_BIAS_RES && (sizeof(TO) == 2 || SPLIT)), "LN statistics");
    static_assert(!LN_IN || ((EPI == CLIPK_EPI_BIAS || epi_qgelu(EPI)) && (sizeof(T) == 2 || SPLIT)), "LN fold");
    [[maybe_unused]] f32x2 lnp[LN_IN ? 2 : 1][NQ];
    [[maybe_unused]] f32x2 lnpart[LN_MERGE ? TM : 1][NQ];
    auto load_ln = [&](int i, int slot) {
      if constexpr (LN_IN && !LN_MERGE) {
        const int mg = m0 + wm * (BM / WM) + i * 16;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          int mc = mg + RPQ * q + er;
          mc = mc < g.M ? mc : g.M - 1;
          lnp[slot][q] = g.lnrnb[mc];  // one 8-B load per row
        }
      }
    };
    if (stp && ti < STAMP_TILES) stp[2 + 3 * ti] = __builtin_amdgcn_s_memrealtime();
    if constexpr (PP) {
      constexpr int TM2 = TM / 2, TN2 = TN / 2;
      constexpr int HA = BM / 32;        // 8-row units of one wave row's A half (BM/4 rows)
      constexpr int UA = 2 * HA, UB = 16;  // units per A / B region
      constexpr int NA_HI = UA - NW;     // waves w < NA_HI issue 2 units of an A region, others 1
      static_assert(UA >= NW && UA <= 2 * NW && UB == 2 * NW, "region split");
      // region r: 0 = A half 0, 1 = A half 1, 2 = B half 0, 3 = B half 1; unit u = w + NW*i
      // (wave-uniform first row row0, a multiple of 8). A lane stages row row0 + lrow, 16-B
      // chunk (lane % 8) ^ swz(row) = lco ^ (row0 & 8 ? 4 : 0) chunks, by buffer LDS-DMA: the
      // lane's byte offset within its tile is tile-independent (poff) and the tile enters as
      // the resource base, whose size drops the rows past M (no clamp, no per-load address math).
      const int lrow = lane / CPR;
      const int lco = ((lane % CPR) ^ (lrow >> 1)) * 16;
      const bool two_a = w < NA_HI;
      auto unit_row0 = [&](int r, int i) {
        const int u = w + NW * i;
        if (r < 2) {
          const int uu = u < UA ? u : 0;
          return (uu / HA) * (BM / 2) + r * (BM / 4) + (uu % HA) * 8;
        }
        return (u / 4) * 64 + (r - 2) * 32 + (u % 4) * 8;
      };
      int poff[4][2];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row0 = unit_row0(r, i);
          poff[r][i] = (row0 + lrow) * (r < 2 ? g.lda : g.ldb) * (int)esz + (lco ^ ((row0 & 8) << 3));
        }
      auto rsrc_a = [&](int tm0) {
        return tile_rsrc(g.A + (size_t)tm0 * g.lda * esz, (long long)(g.M - tm0) * g.lda * (long long)esz);
      };
      auto rsrc_b = [&](int tn0) {
        return tile_rsrc(g.B + (size_t)tn0 * g.ldb * esz, (long long)BN * g.ldb * (long long)esz);
      };
      typedef __amdgpu_buffer_rsrc_t TRes;
      // stage region r of K tile kt into buffer buf from the tile resources ra / rb
      // kt: absolute K tile (the item's kt0c + local index; the next item's kt0n + ...)
      auto pst = [&](int buf, __amdgpu_buffer_rsrc_t ra_, __amdgpu_buffer_rsrc_t rb_, int kt, int r) {
        if (CLIPK_GEMM_NOLOAD && it >= 1) return;  // diagnostic: first K tiles only
        const int base = buf * STAGE;
        const int koff = kt * ROWB;
#pragma unroll
        for (int i = 0; i < 2; ++i)
          if (r >= 2 || i == 0 || two_a) {
            const int row0 = unit_row0(r, i);
            if (CLIPK_GEMM_APOL != 0 && r < 2)
              __builtin_amdgcn_raw_ptr_buffer_load_lds(
                  ra_, (__attribute__((address_space(3))) void*)(smem + base + row0 * ROWB), 16, poff[r][i], koff, 0,
                  CLIPK_GEMM_APOL);
            else
              __builtin_amdgcn_raw_ptr_buffer_load_lds(
                  r < 2 ? ra_ : rb_, (__attribute__((address_space(3))) void*)(smem + base + (r < 2 ? 0 : OPA) + row0 * ROWB),
                  16, poff[r][i], koff, 0, 0);
          }
      };
      // K step s+1 landed; the three regions already issued for s+2 (A0, B1, A1) stay in flight
      // (+ the warm-up load issued between B1 and A1, CLIPK_GEMM_WARM)
      constexpr bool WARM = CLIPK_GEMM_WARM > 0 && BM == 192 && !SPLIT;
      const bool warm_w = WARM && w < BM / 64;
      auto wait_ahead = [&]() {
        if (warm_w) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
        else if (two_a) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      };
      // one dword of A row (w * 64 + lane) of the tile at K tile kw: its 128-B line into L2, by an
      // LDS-DMA into a junk area (no register result, so no compiler wait; wait_ahead counts it)
      auto warm = [&](__amdgpu_buffer_rsrc_t ra_, int kw) {
        if constexpr (WARM) {
          if (warm_w)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                ra_, (__attribute__((address_space(3))) void*)(smem + DEPTH * STAGE + NW * EPI_SCRATCH + w * 256), 4,
                (w * 64 + lane) * g.lda * (int)esz, kw * ROWB, 0, 0);
        }
      };
      constexpr int NFB = CLIPK_GEMM_PPB0 ? 2 : 1;
      u32x4 fa[KK][TM2], fbs[NFB][KK][TN2];
      int kga = 0;  // LNM 4: the absolute K step whose A fragments rd_a reads
      [[maybe_unused]] f32x4 gam[2];
      auto rd_a = [&](int buf, int h) {
        const char* As = smem + buf * STAGE + (wm * (BM / WM) + h * (BM / WM / 2) + fr) * ROWB;
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
#pragma unroll
          for (int i = 0; i < TM2; ++i)
            fa[kk][i] = *reinterpret_cast<const u32x4*>(As + i * 16 * ROWB + (((SPLIT ? 2 * fq + kk : kk * 4 + fq)) ^ sw) * 16);
        if constexpr (LN_GAMMA) {  // gamma of the lane's 8 k (chunks 2 fq, 2 fq + 1 of the step)
          gam[0] = *reinterpret_cast<const f32x4*>(sgam + kga * 32 + 8 * fq);
          gam[1] = *reinterpret_cast<const f32x4*>(sgam + kga * 32 + 8 * fq + 4);
        }
      };
      auto rd_b = [&](int buf, int q) {
        const char* Bs = smem + buf * STAGE + OPA + (wn * (BN / WN) + q * (BN / WN / 2) + fr) * ROWB;
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
#pragma unroll
          for (int j = 0; j < TN2; ++j)
            fbs[NFB == 2 ? q : 0][kk][j] =
                *reinterpret_cast<const u32x4*>(Bs + j * 16 * ROWB + (((SPLIT ? 2 * fq + kk : kk * 4 + fq)) ^ sw) * 16);
      };
      auto mm = [&](int h, int q) {
        if (CLIPK_GEMM_NOMMA) return;
        if (CLIPK_GEMM_PRIO == 1) __builtin_amdgcn_s_setprio(1);
        if constexpr (SPLIT) {  // fa[0][i] / fa[1][i]: the A half's hi / lo parts (split_a)
#pragma unroll
          for (int i = 0; i < TM2; ++i)
#pragma unroll
            for (int j = 0; j < TN2; ++j)
              acc[h * TM2 + i][q * TN2 + j] = mma_split<TWO_TERMS, W16>(fbs[NFB == 2 ? q : 0][0][j], fbs[NFB == 2 ? q : 0][1][j],
                                                        fa[0][i], fa[1][i], acc[h * TM2 + i][q * TN2 + j]);
        } else {
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
#pragma unroll
          for (int i = 0; i < TM2; ++i)
#pragma unroll
            for (int j = 0; j < TN2; ++j)
              acc[h * TM2 + i][q * TN2 + j] = mma<T>(fbs[NFB == 2 ? q : 0][kk][j], fa[kk][i], acc[h * TM2 + i][q * TN2 + j]);
        }
        if (CLIPK_GEMM_PRIO == 1) __builtin_amdgcn_s_setprio(0);
      };
      // PREC fp32s: an A half just read is split into its hi / lo parts in place, once for both
      // B quadrants it meets, in the memory segment (beside the partner wave's MFMAs)
      auto split_a = [&]() {
        if constexpr (SPLIT) {
#pragma unroll
          for (int i = 0; i < TM2; ++i) {
            if constexpr (LN_GAMMA) {
              fa[0][i] = __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, fa[0][i]) * gam[0]);
              fa[1][i] = __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, fa[1][i]) * gam[1]);
            }
            split8(fa[0][i], fa[1][i], fa[0][i], fa[1][i]);
          }
          // wait states after the asm split's VGPR writes, independent of the barrier that
          // follows (A/B knob CLIPK_PP_SPLIT_NOP; see split8)
          if constexpr (CLIPK_PP_SPLIT_NOP > 0) asm volatile("s_nop %0" ::"n"(CLIPK_PP_SPLIT_NOP - 1));
        }
      };
      auto seg_end = [&](bool new_a = false) {  // memory segment done: fragments in registers, then the barrier
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (new_a) split_a();
        if (CLIPK_GEMM_PRIO == 2) __builtin_amdgcn_s_setprio(0);
        G8_BAR();
      };
      // The K steps of this block's tiles form one stream (step `it`, buffer it & 1): the
      // restages for steps s+1 / s+2 reach into the next tile, so its first two K tiles load
      // during this tile's last phases and epilogue (nk >= 2).
      const bool lag = wm == 1;
      const TRes cra = rsrc_a(m0), crb = rsrc_b(n0);
      if constexpr (LN_MERGE) {  // this tile's rows' partials, in flight through the K loop
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            int mc = m0 + wm * (BM / WM) + i * 16 + RPQ * q + er;
            mc = mc < g.M ? mc : g.M - 1;
            lnpart[i][q] = reinterpret_cast<const f32x2*>(g.lnstats)[(size_t)mc * LPR + ec];
          }
      }
      // PP2: K tile t+1 landed; the A0 + B0 regions just issued for t+2 stay in flight
      auto wait_ahead2 = [&]() {
        if (two_a) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      };
      constexpr bool PP2 = CLIPK_GEMM_PP2 == 1 || (CLIPK_GEMM_PP2 == 2 && BM == 256);
      static_assert(!PP2 || NFB == 2, "PP2 keeps all of B's fragments");
      if (it == 0) {
        const int q0 = kt0c, q1 = kt0c + 1;
        if constexpr (PP2) {
          pst(0, cra, crb, q0, 0); pst(0, cra, crb, q0, 2); pst(0, cra, crb, q0, 1); pst(0, cra, crb, q0, 3);
          pst(1, cra, crb, q1, 0); pst(1, cra, crb, q1, 2);
          wait_ahead2();
        } else {
          pst(0, cra, crb, q0, 0); pst(0, cra, crb, q0, 2); pst(0, cra, crb, q0, 1); pst(0, cra, crb, q0, 3);
          pst(1, cra, crb, q1, 0); pst(1, cra, crb, q1, 3); pst(1, cra, crb, q1, 1);
          wait_ahead();
        }
        G8_BAR();
      }
      if (lag) G8_BAR();  // wave row 1 runs one segment behind
      const TRes xra = rsrc_a(has_next ? (next / ntn) * BM : m0);
      const TRes xrb = rsrc_b(has_next ? (next % ntn) * BN : n0);
      if constexpr (PP2)
      for (int kt = 0; kt < nkc; ++kt, ++it) {
        const int b = it & 1;
        kga = kt0c + kt;
        const bool in1 = kt + 1 < nkc, in2 = kt + 2 < nkc;
        const bool h1 = in1 || has_next, h2 = in2 || has_next;
        const int k1 = in1 ? kt0c + kt + 1 : kt0n + kt + 1 - nkc, k2 = in2 ? kt0c + kt + 2 : kt0n + kt + 2 - nkc;
        const TRes ra1 = in1 ? cra : xra, rb1 = in1 ? crb : xrb;
        const TRes ra2 = in2 ? cra : xra, rb2 = in2 ? crb : xrb;
        if (CLIPK_GEMM_PRIO == 2) __builtin_amdgcn_s_setprio(1);
        rd_a(b, 0); rd_b(b, 0); rd_b(b, 1);     // phase 1: A0 x B
        if (h1) {
          pst(b ^ 1, ra1, rb1, k1, 1);
          pst(b ^ 1, ra1, rb1, k1, 3);
        }
        if (!in1) {
          load_ext(0, extq[0]);
          load_ln(0, 0);
        }
        seg_end(true);
        mm(0, 0);
        mm(0, 1);
        G8_BAR();
        if (CLIPK_GEMM_PRIO == 2) __builtin_amdgcn_s_setprio(1);
        rd_a(b, 1);                             // phase 2: A1 x B
        if (h2) {
          pst(b, ra2, rb2, k2, 0);
          pst(b, ra2, rb2, k2, 2);
          wait_ahead2();
        } else if (h1) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        seg_end(true);
        mm(1, 0);
        mm(1, 1);
        G8_BAR();
      }
      else
      for (int kt = 0; kt < nkc; ++kt, ++it) {
        const int b = it & 1;
        kga = kt0c + kt;
        const bool in1 = kt + 1 < nkc, in2 = kt + 2 < nkc;
        const bool h1 = in1 || has_next, h2 = in2 || has_next;
        const int k1 = in1 ? kt0c + kt + 1 : kt0n + kt + 1 - nkc, k2 = in2 ? kt0c + kt + 2 : kt0n + kt + 2 - nkc;
        if (CLIPK_GEMM_PRIO == 2) __builtin_amdgcn_s_setprio(1);
        rd_a(b, 0); rd_b(b, 0);                 // phase 1: A0 x B0
        if (h1) pst(b ^ 1, cra, in1 ? crb : xrb, k1, 2);
        if (!in1) {
          load_ext(0, extq[0]);
          load_ln(0, 0);
        }
        seg_end(true);
        mm(0, 0);
        G8_BAR();
        if (CLIPK_GEMM_PRIO == 2) __builtin_amdgcn_s_setprio(1);
        rd_b(b, 1);                             // phase 2: A0 x B1
        if (h2) pst(b, in2 ? cra : xra, crb, k2, 0);
        seg_end();
        mm(0, 1);
        G8_BAR();
        if (CLIPK_GEMM_PRIO == 2) __builtin_amdgcn_s_setprio(1);
        rd_a(b, 1);                             // phase 3: A1 x B1
        if (h2) {
          pst(b, cra, in2 ? crb : xrb, k2, 3);
          // the warm-up rides between B1 and A1 of s+2 (wait_ahead counts it): this tile's A
          // CLIPK_GEMM_WARM steps ahead, clamped to its last K tile
          warm(cra, kt0c + min(kt + CLIPK_GEMM_WARM, nkc - 1));
        }
        seg_end(true);
        mm(1, 1);
        G8_BAR();
        if (CLIPK_GEMM_PRIO == 2) __builtin_amdgcn_s_setprio(1);
        if (NFB == 1) rd_b(b, 0);               // phase 4: A1 x B0
        if (h2) {
          pst(b, in2 ? cra : xra, crb, k2, 1);
          wait_ahead();
        } else if (h1) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        seg_end();
        mm(1, 0);
        G8_BAR();
      }
      if (!lag) G8_BAR();  // both wave rows level again: the epilogues run side by side
    } else
    // group 0's operands are loaded at the top of the last K step (its MFMAs hide them)
    for (int kt = 0; kt < nk; ++kt, ++it) {
      const int cur = DEPTH == 2 ? (it & 1) : it % DEPTH;
      const bool last = kt + 1 == nk;
      if constexpr (DEPTH == 2) {
        if (!last) {
          stage(cur ^ 1, kt + 1);
        } else if (has_next) {
          set_tile(next);
          stage(cur ^ 1, 0);  // next tile's first stage flies during this tile's epilogue
        }
      } else {
        if (kt + DEPTH - 1 < nk) stage((kt + DEPTH - 1) % DEPTH, kt + DEPTH - 1);  // slot read at kt-1
      }
      if (last) {
        load_ext(0, extq[0]);
        load_ln(0, 0);
      }
      const char* As = smem + cur * STAGE + (wm * (BM / WM) + fr) * ROWB;
      const char* Bs = smem + cur * STAGE + OPA + (wn * (BN / WN) + fr) * ROWB;
      if constexpr (SPLIT) {
        const int p0 = ((2 * fq) ^ sw) * 16, p1 = ((2 * fq + 1) ^ sw) * 16;
        u32x4 bh[TN], bl[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          bh[j] = *reinterpret_cast<const u32x4*>(Bs + j * 16 * ROWB + p0);
          bl[j] = *reinterpret_cast<const u32x4*>(Bs + j * 16 * ROWB + p1);
        }
        [[maybe_unused]] f32x4 gm0, gm1;
        if constexpr (LN_GAMMA) {
          gm0 = *reinterpret_cast<const f32x4*>(sgam + (kt0 + kt) * 32 + 8 * fq);
          gm1 = *reinterpret_cast<const f32x4*>(sgam + (kt0 + kt) * 32 + 8 * fq + 4);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          u32x4 ah, al, x0 = *reinterpret_cast<const u32x4*>(As + i * 16 * ROWB + p0),
                        x1 = *reinterpret_cast<const u32x4*>(As + i * 16 * ROWB + p1);
          if constexpr (LN_GAMMA) {
            x0 = __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, x0) * gm0);
            x1 = __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, x1) * gm1);
          }
          split8<false>(x0, x1, ah, al);  // MFMAs follow within a few instructions
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma_split<TWO_TERMS, W16>(bh[j], bl[j], ah, al, acc[i][j]);
        }
      } else
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int p = ((kk * 4 + fq) ^ sw) * 16;
        u32x4 a[TM], b[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = *reinterpret_cast<const u32x4*>(Bs + j * 16 * ROWB + p);
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = *reinterpret_cast<const u32x4*>(As + i * 16 * ROWB + p);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma<T>(b[j], a[i], acc[i][j]);
      }
      if (!last) {
        if constexpr (DEPTH == 2) {
          write_a(cur ^ 1);  // AG: slot cur^1 was last read in step kt-1 (before its barrier)
          if (!CLIPK_GEMM_NOBAR) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
          }
        } else {
          ring_wait(min(DEPTH - 2, nk - 2 - kt));  // stages kt+2 .. issued after kt+1
          G8_BAR();
        }
      }
    }

    // ---- epilogue through a per-wave LDS scratch [16][64] fp32: the MFMA layout (lane =
    // row fr, 4 columns per sub-tile) is transposed to row-major so that each store / residual
    // / aux access instruction covers 4 rows x full 64-column runs (128 B of f16, 256 B of
    // f32) instead of 16 rows x 32 B. 16-B chunk c of row r sits at chunk c ^ r (conflict-free
    // on both the write and the read-back side).
    if (stp && ti < STAMP_TILES) stp[3 + 3 * ti] = __builtin_amdgcn_s_memrealtime();
    static_assert(TN == 4, "epilogue assumes 64 columns per wave");
    float bia[CW];
#pragma unroll
    for (int c = 0; c < CW; ++c) bia[c] = 0.f;
    if constexpr (HAS_BIAS) {
#pragma unroll
      for (int c = 0; c < CW; c += 4) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(g.bias + ncol + c);
        bia[c] = b4[0]; bia[c + 1] = b4[1]; bia[c + 2] = b4[2]; bia[c + 3] = b4[3];
      }
    }
    [[maybe_unused]] float csum[LN_IN ? CW : 1];
    if constexpr (LN_IN) {
#pragma unroll
      for (int c = 0; c < CW; c += 4) {
        const f32x4 s4 = *reinterpret_cast<const f32x4*>(g.colsum + ncol + c);
        csum[c] = s4[0]; csum[c + 1] = s4[1]; csum[c + 2] = s4[2]; csum[c + 3] = s4[3];
      }
      if (TM > 1) load_ln(1, 1);
    }
    float* scr = reinterpret_cast<float*>(smem + DEPTH * STAGE + w * EPI_SCRATCH);
    const long long rows_ok = (long long)(g.M - m0 < BM ? g.M - m0 : BM);
    // LN statistics: (sum, sum of squares about the group mean) of each row's 64 columns
    // [nbase, nbase + 64), written by the row's first lane (the others store out of range)
    const int lng = g.N / 64;
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t rst =
        tile_rsrc(LN_OUT ? g.lnstats + (size_t)m0 * lng * 2 : nullptr, LN_OUT ? rows_ok * lng * 8 : 0);
    const __amdgpu_buffer_rsrc_t ro = tile_rsrc(outb + (size_t)m0 * g.ldo, rows_ok * g.ldo * (long long)sizeof(TO));
    __amdgpu_buffer_rsrc_t ro2 = ro;
    if constexpr (epi_qgelu(EPI))
      ro2 = tile_rsrc(g.out2 ? (const TO*)g.out2 + (size_t)m0 * g.ldo : nullptr,
                      g.out2 ? rows_ok * g.ldo * (long long)sizeof(TO) : 0);
#pragma unroll
    for (int d = 1; d < XD; ++d) load_ext(d, extq[d]);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int mg = m0 + wm * (BM / WM) + i * 16;  // first row of this 16-row group
      XR ext[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) ext[q] = extq[i % XD][q];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // previous group's read-back done
#pragma unroll
      for (int j = 0; j < TN; ++j)
        *reinterpret_cast<f32x4*>(scr + fr * 64 + (((4 * j + fq) ^ fr) << 2)) = acc[i][j];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private: no barrier needed
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int rr = RPQ * q + er;
        const int m = mg + rr;
        float v[CW];
#pragma unroll
        for (int c = 0; c < CW / 4; ++c) {  // 16-B chunk (CW/4)*ec + c of row rr sits at chunk ^ rr
          const f32x4 t = *reinterpret_cast<const f32x4*>(scr + rr * 64 + ((((CW / 4) * ec + c) ^ rr) << 2));
          v[4 * c] = t[0]; v[4 * c + 1] = t[1]; v[4 * c + 2] = t[2]; v[4 * c + 3] = t[3];
        }
        const int off = ((m - m0) * g.ldo + ncol) * (int)sizeof(TO);  // rows >= M: out of range, dropped
        if constexpr (SPLIT) {
#pragma unroll
          for (int c = 0; c < CW; ++c) v[c] *= kSplitAlpha;  // exact (power of 2)
        }
        if constexpr (LN_MERGE) {
          // clipk_ln_stats_merge's arithmetic on the row's 8 partials (ln_stats_merge_kernel)
          const f32x2 pp = lnpart[i][q];
          const float mu = sum8(pp[0]) * (1.0f / 512.0f);
          const float d = pp[0] * (1.0f / 64.0f) - mu;
          const float rs = rsqrtf(sum8(fmaf(64.0f * d, d, pp[1])) * (1.0f / 512.0f) + 1e-5f);
          const float nb = -rs * mu;
          if (n0 == 0 && ec == 0 && m < g.M) {
            if (g.lnmean) g.lnmean[m] = mu;
            if (g.lnrstd) g.lnrstd[m] = rs;
            g.lnrnb_out[m] = (f32x2){rs, nb};
          }
#pragma unroll
          for (int c = 0; c < CW; ++c) v[c] = fmaf(rs, v[c], fmaf(nb, csum[c], bia[c]));
        } else if constexpr (LN_IN) {
          const float rs = lnp[i & 1][q][0], nb = lnp[i & 1][q][1];
#pragma unroll
          for (int c = 0; c < CW; ++c) v[c] = fmaf(rs, v[c], fmaf(nb, csum[c], bia[c]));
        } else if constexpr (HAS_BIAS) {
#pragma unroll
          for (int c = 0; c < CW; ++c) v[c] += bia[c];
        }
        if constexpr (EPI == CLIPK_EPI_BIAS_RES) {
          float r[CW];
          raw_f32<TX, CW>(ext[q], r);
#pragma unroll
          for (int c = 0; c < CW; ++c) v[c] += r[c];
          if constexpr (LN_OUT) {
            float vr[CW], s = 0.f, s2 = 0.f;
#pragma unroll
            for (int c = 0; c < CW; ++c) {
              vr[c] = to_f32((TO)v[c]);  // the stored value
              s += vr[c];
            }
            s = sum_group<LPR>(s);
            const float mu = s * (1.0f / 64.0f);
#pragma unroll
            for (int c = 0; c < CW; ++c) {
              const float d = vr[c] - mu;
              s2 = fmaf(d, d, s2);
            }
            s2 = sum_group<LPR>(s2);
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            const int so = ec == 0 ? ((m - m0) * lng + nbase / 64) * 8 : 0x40000000;
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, (f32x2){s, s2}), rst, so, 0, 0);
          }
        } else if constexpr (EPI == CLIPK_EPI_BIAS_QGELU) {
          buf_store16<TO>(ro2, off, v);  // no-op when out2 is null (zero-sized resource)
#pragma unroll
          for (int c = 0; c < CW; ++c) v[c] = quick_gelu(v[c]);
        } else if constexpr (EPI == EPI_QGELU_D) {
          // the derivative from the same sigmoid: 3 more VALU per element here, and the
          // backward's epilogue (EPI_DMUL) is one multiply instead of exp + rcp + 6
          float dq[CW];
#pragma unroll
          for (int c = 0; c < CW; ++c) {
            const float sg = qgelu_sigmoid(v[c]);
            dq[c] = sg * fmaf(1.702f * v[c], 1.0f - sg, 1.0f);
            v[c] *= sg;
          }
          buf_store16<TO>(ro2, off, dq);
        } else if constexpr (EPI == CLIPK_EPI_DQGELU) {
          float h[CW];
          raw_f32<TX, CW>(ext[q], h);
#pragma unroll
          for (int c = 0; c < CW; ++c) v[c] *= quick_gelu_grad(h[c]);
        } else if constexpr (EPI == EPI_DMUL) {
          float dq[CW];
          raw_f32<TX, CW>(ext[q], dq);
#pragma unroll
          for (int c = 0; c < CW; ++c) v[c] *= dq[c];
        }
        constexpr bool CHAIN = epi_qgelu(EPI) || EPI == CLIPK_EPI_DQGELU || EPI == EPI_DMUL;
        buf_store16<TO, LN_OUT ? CLIPK_GEMM_SPOL_LN : (CHAIN ? CLIPK_GEMM_SPOL_CHAIN : CLIPK_GEMM_SPOL)>(ro, off, v);
      }
      if (i + XD < TM) load_ext(i + XD, extq[i % XD]);  // this group's slot is free again
      if (i + 2 < TM) load_ln(i + 2, i & 1);
    }
    if (stp && ti < STAMP_TILES) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stp[4 + 3 * ti] = __builtin_amdgcn_s_memrealtime();
    }
    ++ti;
    if (!has_next) {
      if (stp) { stp[2 + 3 * STAMP_TILES] = __builtin_amdgcn_s_memtime(); stp[3 + 3 * STAMP_TILES] = __builtin_amdgcn_s_memrealtime(); }
      break;
    }
    tile = next;
    if constexpr (!PP) {
      // the K loop left `it` one past this tile's last step: buffer it & 1 holds the
      // next tile's prefetched first stage
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
}


// Tile configurations: 0 = 128x128 (4 waves, 64 KiB LDS, 2 blocks/CU),
// 1 = 256x256 (8 waves, 128 KiB, persistent when the grid exceeds 2 waves of CUs),
// 2 = 256x128 (8 waves, 96 KiB), 3 = 256x256 non-persistent (benchmark knob),
// 6 = 192x256 (8 waves of 96x64, 112 KiB + scratch): 4/3 more row tiles, chosen when it
// fills the last wave of CUs better than 256-row tiles (N = 512 at 47k rows: 1.45 -> 1.92
// waves).
static int g_force_cfg = -2;  // -2: unread, -1: auto
static int num_cus();
static int pick_cfg(int M, int N, int esz) {
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
static unsigned long long* gemm_stamp_buf() {
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
static bool deep_small() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLIPK_GEMM_DEEP");
    v = e ? atoi(e) : 1;
  }
  return v != 0;
}

static int g_skew = -1;
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

// ping-pong launches: one block per CU at most, a multiple of 8 (XCD groups of the tile split)
[[maybe_unused]] static int pp_grid(int nwg, int cus) {
  const int full = (cus / 8) * 8;
  const int need = (nwg + 7) / 8 * 8;
  if (CLIPK_GEMM_PP == 2) return need;  // one tile per block (A/B)
  return need < full ? need : full;
}

// BM x 256 ping-pong launch when built in and the shape has >= 2 K tiles (the 256-row forms
// with an fp32 residual / aux operand would spill: they keep the 2-slot loop)
template <typename T, typename TO, typename TX, int EPI, int BM, int LNM = 0>
static bool try_pp(const GemmArgs& g, int nwg, hipStream_t st) {
  constexpr bool ext32 = (EPI == CLIPK_EPI_BIAS_RES || EPI == CLIPK_EPI_DQGELU || EPI == EPI_DMUL) && sizeof(TX) == 4;
  if constexpr (CLIPK_GEMM_PP && (sizeof(T) == 2 || is_split_v<T>) && !(BM == 256 && ext32)) {
    if (g.K * (int)sizeof(T) < 2 * GEMM_ROWB) return false;
    hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, BM, 256, 2, 4, true, GEMM_ROWB, 2, false, true, LNM>),
                       dim3(pp_grid(nwg, num_cus())), dim3(512), 0, st, g);
    return true;
  }
  return false;
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

// PREC fp32s (CLIPK_F32S) launches: fp32 out / residual / aux. Large M (where the 16-bit policy
// picks the 192- or 256-row tiles): the ping-pong loop on 192x256 tiles (256-row ones spill at
// 256 VGPRs with the split's temporaries); otherwise 128x128 tiles (a 4-slot ring when the grid
// is at most one tile per CU).
// (Until the split8 hazard above was found, CLIPK_F32S16 ran the 2-MFMA kernel on the ping-pong
// tiles only: on the 2- / 4-slot loop it measured not bit-identical. With the compiler-visible
// split there it is bitwise the 3-MFMA kernel on every tile path, profiles/r05w16/hazard.txt.)
template <int EPI, int LNM = 0, typename TS = f32s>
static int launch_gemm_split(const GemmArgs& g, hipStream_t st) {
  const int cus = num_cus();
  const_cast<GemmArgs&>(g).stamp = gemm_stamp_buf();
  const_cast<GemmArgs&>(g).skew = 0;
  const int cfg = pick_cfg(g.M, g.N, 2);
  if (cfg == 7) {  // small M (the ViT): 64x128 tiles, twice the 128x128 grid
    const int nwg = ((g.M + 63) / 64) * (g.N / 128);
    if (nwg <= cus && deep_small())
      hipLaunchKernelGGL((gemm_nt_kernel<TS, float, float, EPI, 64, 128, 2, 2, false, GEMM_ROWB, 4, false, false, LNM>), dim3(nwg),
                         dim3(256), 0, st, g);
    else
      hipLaunchKernelGGL((gemm_nt_kernel<TS, float, float, EPI, 64, 128, 2, 2, false, GEMM_ROWB, 2, false, false, LNM>), dim3(nwg),
                         dim3(256), 0, st, g);
    CLIPK_CHECK_LAUNCH();
    return CLIPK_OK;
  }
  if (cfg == 1 || cfg == 6) {
    if (try_pp<TS, float, float, EPI, 192, LNM>(g, ((g.M + 191) / 192) * (g.N / 256), st)) {
      CLIPK_CHECK_LAUNCH();
      return CLIPK_OK;
    }
  }
  const int nwg = ((g.M + 127) / 128) * (g.N / 128);
  if (nwg <= cus && deep_small())
    hipLaunchKernelGGL((gemm_nt_kernel<TS, float, float, EPI, 128, 128, 2, 2, false, GEMM_ROWB, 4, false, false, LNM>), dim3(nwg),
                       dim3(256), 0, st, g);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<TS, float, float, EPI, 128, 128, 2, 2, false, GEMM_ROWB, 2, false, false, LNM>), dim3(nwg),
                       dim3(256), 0, st, g);
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
  epi &= ~(CLIPK_A_QGELU | CLIPK_QGELU_DERIV);
  const bool split = in_dtype == CLIPK_F32S || in_dtype == CLIPK_F32S16;
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

// one pass: *flag = 1 when any |W| >= kSplitPackMax or W is not finite (the pack's output
// would hold an inf / NaN part)
__device__ int g_split_range_flag;
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

extern "C" int clipk_split_pack(int N, int K, const float* W, int ldw, void* out, void* stream) {
  if (!W || !out) return CLIPK_EINVAL;
  if (N <= 0 || K <= 0 || K % 32 != 0 || ldw < K) return CLIPK_ESHAPE;
  // the range precondition is enforced here, not left to the caller: one synchronous check
  // (packing runs once per model, at construction) through a module-scope flag
  {
    const hipStream_t st = (hipStream_t)stream;
    int h = 0;
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_split_range_flag), &h, sizeof(int), 0, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
      int* flag = nullptr;
      e = hipGetSymbolAddress((void**)&flag, HIP_SYMBOL(g_split_range_flag));
      if (e == hipSuccess) {
        const long n = (long)N * K, nb = (n + 255) / 256;
        hipLaunchKernelGGL(split_range_kernel, dim3((unsigned)(nb < 1024 ? nb : 1024)), dim3(256), 0, st, N, K, W, ldw,
                           flag);
        e = hipGetLastError();
      }
    }
    if (e == hipSuccess)
      e = hipMemcpyFromSymbolAsync(&h, HIP_SYMBOL(g_split_range_flag), sizeof(int), 0, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return (int)e;
    if (h) return CLIPK_ERANGE;
  }
  const long n = (long)N * (K / 8);
  hipLaunchKernelGGL(split_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, N, K, W,
                     ldw, (f16*)out);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

// *flag = 1 when any lo part of a packed weight is nonzero (per 8 k: 16 B hi, then 16 B lo)
__device__ int g_split_lo_flag;
__global__ __launch_bounds__(256) void split_lo_kernel(long ngroups, const u32x4* __restrict__ packed,
                                                       int* __restrict__ flag) {
  bool nz = false;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < ngroups; i += (long)gridDim.x * 256) {
    const u32x4 lo = packed[2 * i + 1];
    nz |= ((lo[0] | lo[1] | lo[2] | lo[3]) & 0x7fff7fffu) != 0;  // -0 counts as zero
  }
  if (__any(nz) && (threadIdx.x & 63) == 0) *flag = 1;
}

extern "C" int clipk_split_lo_zero(int N, int K, const void* packed, void* stream) {
  if (!packed) return CLIPK_EINVAL;
  if (N <= 0 || K <= 0 || K % 32 != 0) return CLIPK_ESHAPE;
  const hipStream_t st = (hipStream_t)stream;
  int h = 0;
  int* flag = nullptr;
  hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_split_lo_flag), &h, sizeof(int), 0, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipGetSymbolAddress((void**)&flag, HIP_SYMBOL(g_split_lo_flag));
  if (e == hipSuccess) {
    const long ng = (long)N * (K / 8), nb = (ng + 255) / 256;
    hipLaunchKernelGGL(split_lo_kernel, dim3((unsigned)(nb < 1024 ? nb : 1024)), dim3(256), 0, st, ng,
                       (const u32x4*)packed, flag);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyFromSymbolAsync(&h, HIP_SYMBOL(g_split_lo_flag), sizeof(int), 0, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return (int)e;
  return h ? 0 : 1;
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
  epi &= ~CLIPK_QGELU_DERIV;
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
  if (in_dtype == CLIPK_F32S) return dispatch_ln_split<f32s>(epi, g, st);
  if (in_dtype == CLIPK_F32S16) return dispatch_ln_split<f32h>(epi, g, st);
  return in_dtype == CLIPK_F16 ? dispatch_ln<f16>(epi, g, st) : dispatch_ln<bf16>(epi, g, st);
}

// the fold with the LayerNorm weight on A (LNM 4; include/clipk.h): PREC fp32s only
extern "C" int clipk_gemm_ln_gamma(int in_dtype, int epi, int M, int N, int K, const void* A, int lda, const void* B,
                                   int ldb, const float* bias, void* out, int ldo, void* out2, const float* colsum,
                                   const float* rnb, const float* gamma, void* stream) {
  if (!A || !B || !out || !bias || !colsum || !rnb || !gamma) return CLIPK_EINVAL;
  if (in_dtype != CLIPK_F32S && in_dtype != CLIPK_F32S16) return CLIPK_EDTYPE;
  const bool deriv = (epi & CLIPK_QGELU_DERIV) != 0;
  epi &= ~CLIPK_QGELU_DERIV;
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
