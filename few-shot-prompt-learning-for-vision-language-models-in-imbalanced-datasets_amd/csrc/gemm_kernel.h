// gemm_kernel.h -- the MFMA GEMM kernel template and its launch helpers, shared by gemm.hip (the
// C-ABI entry points and the plain instantiations) and gemm_presplit.hip (the PREC fp32s launches
// with pre-split operands, compiled as their own translation unit).
#pragma once
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
// The 8 v_fma_mix of a split are ONE inline-asm statement that ends with its own wait states:
// hipcc's hazard recognizer does not see the VGPRs an asm statement writes, and the ISA rule for
// a VALU write of a VGPR that an MFMA then reads as SrcA / SrcB is 2 wait states (the guide's
// inline-asm rule, cdna_hip_programming.md §5.7 item 2: "a just-written "v" operand -> MFMA
// operand (s_nop 1)"; hipcc applies the same rule to the compiler-visible form of this sequence:
// the v_fma_mixhi_f16 -> v_mfma_f32_16x16x32_f16 pair gets its s_nop, tools/lab/split_hazard.hip).
// With `s_nop 1` inside the string the parts are safe for any consumer hipcc schedules after
// the statement, so no caller counts wait states (round 5 counted them by hand: an MFMA two
// instructions after the split read stale parts, off by up to 5.8e-2, profiles/r05w16/hazard.txt).
#ifndef CLIPK_SPLIT_MIX
#define CLIPK_SPLIT_MIX 1
#endif
__device__ __forceinline__ void split_lo8(const f32x4& x0, const f32x4& x1, const u32x4& hi, u32x4& lo) {
  unsigned l0, l1, l2, l3;
  asm("v_fma_mixlo_f16 %0, %4, 1.0, -%12 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %5, 1.0, -%12 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %1, %6, 1.0, -%13 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %7, 1.0, -%13 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %2, %8, 1.0, -%14 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %2, %9, 1.0, -%14 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %3, %10, 1.0, -%15 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %3, %11, 1.0, -%15 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "s_nop 1"
      : "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3)
      : "v"(x0[0]), "v"(x0[1]), "v"(x0[2]), "v"(x0[3]), "v"(x1[0]), "v"(x1[1]), "v"(x1[2]), "v"(x1[3]),
        "v"(hi[0]), "v"(hi[1]), "v"(hi[2]), "v"(hi[3]));
  lo = (u32x4){l0, l1, l2, l3};
}
// MIX false: the lo part in compiler-visible cvt + sub + cvt form (A/B knob CLIPK_SPLIT_MIX=0).
template <bool MIX = CLIPK_SPLIT_MIX != 0>
__device__ __forceinline__ void split8(u32x4 a0, u32x4 a1, u32x4& hi, u32x4& lo) {
  // the inputs as materialised fp32 values: a caller's x * gamma (the fold's LayerNorm weight) must
  // not contract with the x - hi below into one fma (the parts of the unrounded product), so every
  // path -- this one, the asm form, a producer's pre-split store -- splits the same rounded value
  asm volatile("" : "+v"(a0), "+v"(a1));
  const f32x4 x0 = __builtin_bit_cast(f32x4, a0), x1 = __builtin_bit_cast(f32x4, a1);
  f16x8 h;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    h[c] = (f16)x0[c];
    h[4 + c] = (f16)x1[c];
  }
  hi = __builtin_bit_cast(u32x4, h);
  if constexpr (!MIX) {
    f16x8 l;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      l[c] = (f16)(x0[c] - (float)h[c]);
      l[4 + c] = (f16)(x1[c] - (float)h[4 + c]);
    }
    lo = __builtin_bit_cast(u32x4, l);
    return;
  }
  split_lo8(x0, x1, hi, lo);
}
// a . b ~= hi(a) hi(b) + hi(a) lo(b) + lo(a) hi(b) (lo . lo ~ 2^-22 relative is dropped); the
// weight's parts (packed, clipk_split_pack) are the instruction's A operand (swapped operands)
// Precision experiment (build-time, A/B only): CLIPK_SPLIT_TERMS 2 drops the
// lo(a) hi(b) term -- the activation operand rounded to fp16, the weight kept at ~22 bits -- in
// the GEMMs of epilogue class `CLIPK_SPLIT_TERMS_EPI` (0: every GEMM, 1: the backward's input-grad
// GEMMs, EPI_NONE / EPI_DMUL / EPI_DQGELU).
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
// Split-form epilogue stores form the lo parts by v_fma_mix, and the LayerNorm fold carries the
// weights' scale on the row's rstd (A/B knob: 0 = the convert / subtract form and a multiply per
// element; bitwise the same outputs)
#ifndef CLIPK_EPI_MIXSPLIT
#define CLIPK_EPI_MIXSPLIT 1
#endif
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
// NOSPLIT = the split GEMMs' ping-pong loop takes A's fp32 bits as its hi / lo parts (no split VALU:
// the loop's ceiling without the activation split).
#ifndef CLIPK_GEMM_NOSPLIT
#define CLIPK_GEMM_NOSPLIT 0
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
// SPF (PREC fp32s, split GEMMs): 1 = A is given pre-split (CLIPK_A_SPLIT: the fp16 hi / lo parts of
// each fp32 value, per 8 consecutive k 16 B of hi then 16 B of lo -- the layout the split loop's
// fragments read, so they feed the MFMAs with no split VALU); 2 = the primary output is stored in
// that form (CLIPK_OUT_SPLIT, for a consumer GEMM's A); 4 = EPI_BIAS_RES also stores out2 = that form
// of out * gamma (g.lngamma: the LayerNorm weight of the fold that reads out next,
// CLIPK_OUT2_SPLIT_GAMMA); bits combine.
template <typename T, typename TO, typename TX, int EPI, int BM, int BN, int WM, int WN, bool PERSIST,
          int ROWB = GEMM_ROWB, int DEPTH = 2, bool AG = false, bool PP = false, int LNM = 0, int SPF = 0>
__global__ __launch_bounds__(WM * WN * 64, DEPTH == 2 ? 2 : 1) void gemm_nt_kernel(GemmArgs g) {
  static_assert(DEPTH == 2 || !PERSIST, "deep ring: non-persistent launches only");
  static_assert(!AG || (!PERSIST && DEPTH == 2 && sizeof(T) == 2 && ROWB == 128), "A-operand QuickGELU path");
  // PREC fp32s: 4-byte elements (A fp32, B split-packed), staged as fp32; a 128-B K step is
  // one 32-deep k-window read as two 16-B chunks per fragment (2 fq, 2 fq + 1), 3 MFMAs each
  constexpr bool SPLIT = is_split_v<T>, W16 = __is_same(T, f32h);
  constexpr bool LN_GAMMA = LNM == 4;
  static_assert(!LN_GAMMA || SPLIT, "gamma-on-A fold: split GEMMs");
  // A_PRE with LNM 4: A already holds the split parts of x * gamma (the LayerNorm weight applied by
  // the producer), so the fold's epilogue is LNM 4's with no gamma multiply in the loop
  constexpr bool A_PRE = (SPF & 1) != 0, O_SPLIT = (SPF & 2) != 0, O2_SPLIT = (SPF & 4) != 0;
  static_assert(!O2_SPLIT || (EPI == CLIPK_EPI_BIAS_RES && sizeof(TO) == 4), "split copy of the residual stream");
  constexpr bool GAMMA_A = LN_GAMMA && !A_PRE;  // gamma applied to A's fragments here
  static_assert(!SPF || SPLIT, "pre-split operands: split GEMMs only");
  static_assert(!O_SPLIT || (sizeof(TO) == 4 && EPI != CLIPK_EPI_BIAS_RES), "split-form output: not the residual stream");
  [[maybe_unused]] constexpr bool TWO_TERMS =
      CLIPK_SPLIT_TERMS == 2 && (CLIPK_SPLIT_TERMS_EPI == 0 || EPI == CLIPK_EPI_NONE || EPI == CLIPK_EPI_DQGELU ||
                                 EPI == EPI_DMUL);
  static_assert(!SPLIT || (ROWB == 128 && !AG), "split-fp16 GEMM: 128-B staged rows");
  static_assert(!PP || (PERSIST && !AG && DEPTH == 2 && ROWB == 128 && WM == 2 && WN == 4 && BN == 256 &&
                        (sizeof(T) == 2 || SPLIT) && BM % 64 == 0), "ping-pong main loop (K >= 128)");
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  // B16 (CLIPK_F32S16): B is the compact fp16 weight (clipk_split_hi16: the hi parts of an
  // fp16-valued weight, 2 B per element), so a K step (32 k) of B is a 64-B row: 16 B of the
  // 128-B staged row was the all-zero lo half of each 8-k group. A stays fp32 at 128 B per row.
  // Per 192x256 K step 56 -> 40 KiB staged (B's rows half the bytes).
  constexpr bool B16 = W16;
  constexpr int ROWBB = B16 ? 64 : ROWB;  // bytes per staged B row
  constexpr int OPA = BM * ROWB, OPB = BN * ROWBB, STAGE = OPA + OPB;
  constexpr int RPI = 1024 / ROWB;   // rows per glds wave-instruction (64 lanes x 16 B)
  constexpr int CPR = ROWB / 16;     // 16-B chunks per staged row
  constexpr int RPIB = 1024 / ROWBB, CPRB = ROWBB / 16;  // the same for B's rows
  constexpr int KK = ROWB / 64;      // 64-B MFMA k-windows per K step
  // A stage is NG glds units of RPI rows (1 KiB each, A's GA units then B's), unit g landing
  // at stage offset g * 1024. BLOCKED (every wave the same number of A and of B units): wave w
  // issues A units w*IA.. and B units GA + w*IB..; otherwise units are dealt round-robin
  // (g = w + NW*i) and the first NREM waves issue one more than the others.
  constexpr int GA = BM / RPI, GB = BN / RPIB, NG = GA + GB;
  constexpr bool BLOCKED = GA % NW == 0 && GB % NW == 0;
  constexpr int IA = BLOCKED ? GA / NW : 0, IB = BLOCKED ? GB / NW : 0;
  constexpr int NI = (NG + NW - 1) / NW;  // glds slots per wave (the last may be idle)
  constexpr int PERL = NG / NW, NREM = NG % NW;
  static_assert(ROWB == 128 || (ROWB == 64 && sizeof(T) == 2), "staged row is 128 B (or 64 B for 16-bit)");
  static_assert(BM % RPI == 0 && BN % RPIB == 0 && NG >= NW, "tile/wave mismatch");
  static_assert(!AG || BLOCKED, "A-operand QuickGELU path: blocked unit split");
  // (+ 1 KiB: the CLIPK_GEMM_WARM junk area of the 192-row ping-pong loop)
  constexpr int WARM_B = CLIPK_GEMM_WARM > 0 && PP && BM == 192 ? 1024 : 0;
  constexpr int GAM_OFF = DEPTH * STAGE + NW * EPI_SCRATCH + WARM_B;  // LNM 4: gamma[K] in LDS
  __shared__ CLIPK_LDS_ALIGN char smem[GAM_OFF + (GAMMA_A ? kGammaMax * 4 : 0)];  // one array (see header)
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
  const size_t eszb = B16 ? 2 : esz;  // B's element bytes
  const int nk_all = (int)((size_t)g.K * esz / ROWB);
  const int kt0 = PERSIST ? 0 : ks * nk_all / g.ksplit;
  const int nk = PERSIST ? nk_all : (ks + 1) * nk_all / g.ksplit - kt0;
  TO* const outb = (TO*)g.out + (PERSIST ? 0 : (size_t)ks * g.split_stride);
  // source-side swizzle of 16-B chunk c in row r: 128-B rows c ^ ((r >> 1) & 7), 64-B rows
  // c ^ ((r >> 2) & 3) -- either way 16 consecutive rows read at one chunk hit 16 distinct
  // 16-B slots of the 256-B bank row
  auto swz_rb = [](int r, int rb) { return rb == 128 ? (r >> 1) & 7 : (r >> 2) & 3; };
  auto swz = [&](int r) { return swz_rb(r, ROWB); };
  auto unit = [&](int i) { return BLOCKED ? (i < IA ? w * IA + i : GA + w * IB + (i - IA)) : w + NW * i; };
  auto unit_is_a = [&](int i) { return BLOCKED ? i < IA : unit(i) < GA; };
  const char* src[NI];
  auto set_tile = [&](int t) {
    const int tm0 = (t / ntn) * BM, tn0 = (t % ntn) * BN;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int u = unit(i);
      const bool ua = unit_is_a(i);
      if (ua) {
        const int row = u * RPI + lane / CPR;
        const int c = (lane % CPR) ^ swz(row);  // source-side swizzle
        int ga = tm0 + row;
        ga = ga < g.M ? ga : g.M - 1;
        src[i] = g.A + ((size_t)ga * g.lda) * esz + c * 16 + (size_t)kt0 * ROWB;
      } else {
        const int row = (u - GA) * RPIB + lane / CPRB;
        const int c = (lane % CPRB) ^ swz_rb(row, ROWBB);
        const int gb = u < NG ? tn0 + row : tn0;  // idle slot: a valid address, never issued
        src[i] = g.B + ((size_t)gb * g.ldb) * eszb + c * 16 + (size_t)kt0 * ROWBB;
      }
    }
  };
  u32x4 ra[AG ? IA : 1];  // AG: the next stage's A chunks in flight
  auto stage = [&](int s, int kt) {
    if (CLIPK_GEMM_NOLOAD && kt > 0) return;
    char* base = smem + s * STAGE;
    const size_t koff = (size_t)kt * ROWB, koffb = (size_t)kt * ROWBB;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if constexpr (AG) {
        if (i < IA) {
          ra[i] = *reinterpret_cast<const u32x4*>(src[i] + koff);
          continue;
        }
      }
      const int u = unit(i);
      if (BLOCKED || NREM == 0 || u < NG) glds16(src[i] + (unit_is_a(i) ? koff : koffb), base + u * 1024);
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

  if constexpr (GAMMA_A) {  // the LayerNorm weight, once per block (before any LDS-DMA is issued)
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
      // units per A / B region (B16: a B region is 128 rows x 64 B = 8 units of 16 rows)
      constexpr int UA = 2 * HA, UB = B16 ? 8 : 16;
      constexpr int NA_HI = UA - NW;     // waves w < NA_HI issue 2 units of an A region, others 1
      constexpr int NBR = UB / NW;       // LDS-DMA instructions per wave and B region
      static_assert(UA >= NW && UA <= 2 * NW && (UB == 2 * NW || (B16 && UB == NW)), "region split");
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
        if constexpr (B16) return (u / 2) * 64 + (r - 2) * 32 + (u % 2) * 16;  // 16-row units
        return (u / 4) * 64 + (r - 2) * 32 + (u % 4) * 8;
      };
      // B16: a lane stages row row0 + lane / 4, chunk (lane % 4) ^ ((row >> 2) & 3) of the 64-B
      // row (row0 is a multiple of 16, so the swizzle depends on the lane alone)
      const int lrowb = lane / CPRB;
      const int lcob = ((lane % CPRB) ^ swz_rb(lrowb, ROWBB)) * 16;
      int poff[4][2];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row0 = unit_row0(r, i);
          if (B16 && r >= 2)
            poff[r][i] = (row0 + lrowb) * g.ldb * (int)eszb + lcob;
          else
            poff[r][i] = (row0 + lrow) * (r < 2 ? g.lda : g.ldb) * (int)esz + (lco ^ ((row0 & 8) << 3));
        }
      auto rsrc_a = [&](int tm0) {
        return tile_rsrc(g.A + (size_t)tm0 * g.lda * esz, (long long)(g.M - tm0) * g.lda * (long long)esz);
      };
      auto rsrc_b = [&](int tn0) {
        return tile_rsrc(g.B + (size_t)tn0 * g.ldb * eszb, (long long)BN * g.ldb * (long long)eszb);
      };
      typedef __amdgpu_buffer_rsrc_t TRes;
      // stage region r of K tile kt into buffer buf from the tile resources ra / rb
      // kt: absolute K tile (the item's kt0c + local index; the next item's kt0n + ...)
      auto pst = [&](int buf, __amdgpu_buffer_rsrc_t ra_, __amdgpu_buffer_rsrc_t rb_, int kt, int r) {
        if (CLIPK_GEMM_NOLOAD && it >= 1) return;  // diagnostic: first K tiles only
        const int base = buf * STAGE;
        const int koff = kt * (r < 2 ? ROWB : ROWBB);
#pragma unroll
        for (int i = 0; i < 2; ++i)
          if ((r >= 2 && i < NBR) || (r < 2 && (i == 0 || two_a))) {
            const int row0 = unit_row0(r, i);
            if (CLIPK_GEMM_APOL != 0 && r < 2)
              __builtin_amdgcn_raw_ptr_buffer_load_lds(
                  ra_, (__attribute__((address_space(3))) void*)(smem + base + row0 * ROWB), 16, poff[r][i], koff, 0,
                  CLIPK_GEMM_APOL);
            else
              __builtin_amdgcn_raw_ptr_buffer_load_lds(
                  r < 2 ? ra_ : rb_,
                  (__attribute__((address_space(3))) void*)(smem + base + (r < 2 ? row0 * ROWB : OPA + row0 * ROWBB)),
                  16, poff[r][i], koff, 0, 0);
          }
      };
      // K step s+1 landed; the three regions already issued for s+2 (A0, B1, A1) stay in flight
      // (+ the warm-up load issued between B1 and A1, CLIPK_GEMM_WARM): this wave's LDS-DMAs of
      // those regions, 2 or 1 per A region (two_a) and NBR per B region
      constexpr bool WARM = CLIPK_GEMM_WARM > 0 && BM == 192 && !SPLIT;
      const bool warm_w = WARM && w < BM / 64;
      auto wait_ahead = [&]() {
        if (warm_w) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 + NBR) : "memory");
        else if (two_a) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 + NBR) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 + NBR) : "memory");
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
        if constexpr (GAMMA_A) {  // gamma of the lane's 8 k (chunks 2 fq, 2 fq + 1 of the step)
          gam[0] = *reinterpret_cast<const f32x4*>(sgam + kga * 32 + 8 * fq);
          gam[1] = *reinterpret_cast<const f32x4*>(sgam + kga * 32 + 8 * fq + 4);
        }
      };
      auto rd_b = [&](int buf, int q) {
        const char* Bs = smem + buf * STAGE + OPA + (wn * (BN / WN) + q * (BN / WN / 2) + fr) * ROWBB;
        if constexpr (B16) {  // the hi parts only: chunk fq of the 64-B row (slot 1 unused)
#pragma unroll
          for (int j = 0; j < TN2; ++j) {
            fbs[NFB == 2 ? q : 0][0][j] =
                *reinterpret_cast<const u32x4*>(Bs + j * 16 * ROWBB + ((fq ^ swz_rb(fr, ROWBB)) * 16));
            fbs[NFB == 2 ? q : 0][1][j] = fbs[NFB == 2 ? q : 0][0][j];
          }
          return;
        }
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
        if constexpr (SPLIT && !A_PRE) {  // (A_PRE: the fragments already are the hi / lo parts)
#pragma unroll
          for (int i = 0; i < TM2; ++i) {
            if constexpr (GAMMA_A) {
              fa[0][i] = __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, fa[0][i]) * gam[0]);
              fa[1][i] = __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, fa[1][i]) * gam[1]);
            }
            if constexpr (!CLIPK_GEMM_NOSPLIT) split8(fa[0][i], fa[1][i], fa[0][i], fa[1][i]);
          }
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
        if (two_a) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 + NBR) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 + NBR) : "memory");
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
      const char* Bs = smem + cur * STAGE + OPA + (wn * (BN / WN) + fr) * ROWBB;
      if constexpr (SPLIT) {
        const int p0 = ((2 * fq) ^ sw) * 16, p1 = ((2 * fq + 1) ^ sw) * 16;
        u32x4 bh[TN], bl[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (B16) {  // the lane's 8 k (8 fq ..) are chunk fq of the 64-B row
            bh[j] = *reinterpret_cast<const u32x4*>(Bs + j * 16 * ROWBB + ((fq ^ swz_rb(fr, ROWBB)) * 16));
            bl[j] = bh[j];  // unused (W16: the weight-lo product is not formed)
          } else {
            bh[j] = *reinterpret_cast<const u32x4*>(Bs + j * 16 * ROWB + p0);
            bl[j] = *reinterpret_cast<const u32x4*>(Bs + j * 16 * ROWB + p1);
          }
        }
        [[maybe_unused]] f32x4 gm0, gm1;
        if constexpr (GAMMA_A) {
          gm0 = *reinterpret_cast<const f32x4*>(sgam + (kt0 + kt) * 32 + 8 * fq);
          gm1 = *reinterpret_cast<const f32x4*>(sgam + (kt0 + kt) * 32 + 8 * fq + 4);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          u32x4 ah, al, x0 = *reinterpret_cast<const u32x4*>(As + i * 16 * ROWB + p0),
                        x1 = *reinterpret_cast<const u32x4*>(As + i * 16 * ROWB + p1);
          if constexpr (A_PRE) {
            ah = x0;  // chunk 2 fq: the hi parts of the lane's 8 k, chunk 2 fq + 1 their lo parts
            al = x1;
          } else {
            if constexpr (GAMMA_A) {
              x0 = __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, x0) * gm0);
              x1 = __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, x1) * gm1);
            }
            split8(x0, x1, ah, al);  // (the MFMAs right after it: split_lo8 carries their wait states)
          }
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
    if constexpr (epi_qgelu(EPI) || O2_SPLIT)
      ro2 = tile_rsrc(g.out2 ? (const TO*)g.out2 + (size_t)m0 * g.ldo : nullptr,
                      g.out2 ? rows_ok * g.ldo * (long long)sizeof(TO) : 0);
    // split-form stores (SPF 2 / 4): the 4 fp32 values v of the lane's columns ncol.. of row m as
    // the consumer GEMM's pre-split A -- hi = fp16(v), lo = fp16(v - hi) (v - hi exact in fp32:
    // bitwise the parts that GEMM's own split would form from the fp32 v). Lanes ec and ec ^ 1 hold
    // the two halves of one 8-column group: they swap (DPP quad_perm [1,0,3,2]), then the even lane
    // stores the group's 16 B of hi parts and the odd lane its 16 B of lo parts.
    // keep: plain (cache-kept) stores, as the LN-statistics producers' (CLIPK_GEMM_SPOL_LN); else the
    // chained outputs' policy (CLIPK_GEMM_SPOL_CHAIN)
    [[maybe_unused]] auto store_split = [&](__amdgpu_buffer_rsrc_t rs, int m, const float* v, bool keep) {
      static_assert(CW == 4 || !(O_SPLIT || O2_SPLIT), "split-form output: fp32 epilogue lanes (4 columns)");
      if constexpr (CW == 4) {
        // v - hi must subtract the ROUNDED fp32 v: without the opaque copy the compiler contracts it
        // with v's producing multiply (QuickGELU's x * sigmoid) into one fma -- the parts of the
        // unrounded product, which differ from the consumer's on round-to-even ties (measured)
        float x[4] = {v[0], v[1], v[2], v[3]};
#pragma unroll
        for (int c = 0; c < 4; ++c) asm volatile("" : "+v"(x[c]));
        const f16x2 h01 = {(f16)x[0], (f16)x[1]}, h23 = {(f16)x[2], (f16)x[3]};
        const unsigned hu01 = __builtin_bit_cast(unsigned, h01), hu23 = __builtin_bit_cast(unsigned, h23);
        unsigned l01, l23;  // lo = fp16(x - hi) by v_fma_mix (common.h split_lo4; bitwise the cvt form)
        if constexpr (CLIPK_EPI_MIXSPLIT) {
          split_lo4(x[0], x[1], x[2], x[3], hu01, hu23, l01, l23);
        } else {  // A/B: convert, subtract, convert
          l01 = __builtin_bit_cast(unsigned, (f16x2){(f16)(x[0] - (float)h01[0]), (f16)(x[1] - (float)h01[1])});
          l23 = __builtin_bit_cast(unsigned, (f16x2){(f16)(x[2] - (float)h23[0]), (f16)(x[3] - (float)h23[1])});
        }
        const bool odd = (ec & 1) != 0;
        const int s0 = (int)(odd ? hu01 : l01), s1 = (int)(odd ? hu23 : l23);
        const unsigned r0 = (unsigned)__builtin_amdgcn_update_dpp(0, s0, 0xB1, 0xF, 0xF, false);
        const unsigned r1 = (unsigned)__builtin_amdgcn_update_dpp(0, s1, 0xB1, 0xF, 0xF, false);
        const u32x4 d = odd ? (u32x4){r0, r1, l01, l23} : (u32x4){hu01, hu23, r0, r1};
        const int offs = ((m - m0) * g.ldo + (ncol & ~7)) * 4 + (odd ? 16 : 0);
        if (keep) __builtin_amdgcn_raw_buffer_store_b128(d, rs, offs, 0, CLIPK_GEMM_SPOL_LN);
        else __builtin_amdgcn_raw_buffer_store_b128(d, rs, offs, 0, CLIPK_GEMM_SPOL_CHAIN);
      }
    };
    // SPF 4: the LayerNorm weight of the next fold, for out2 = split(v * gamma)
    [[maybe_unused]] f32x4 g2 = {0.f, 0.f, 0.f, 0.f};
    if constexpr (O2_SPLIT) g2 = *reinterpret_cast<const f32x4*>(g.lngamma + ncol);
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
        // the packed weights' scale undone: exact (a power of 2), so under the LayerNorm fold it
        // rides on the row's rstd (fma(rs * alpha, v, t) == fma(rs, v * alpha, t) bitwise)
        if constexpr (SPLIT && (!LN_IN || !CLIPK_EPI_MIXSPLIT)) {
#pragma unroll
          for (int c = 0; c < CW; ++c) v[c] *= kSplitAlpha;
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
          const float rs = lnp[i & 1][q][0] * (SPLIT && CLIPK_EPI_MIXSPLIT ? kSplitAlpha : 1.0f), nb = lnp[i & 1][q][1];
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
          if constexpr (O2_SPLIT) {  // the next fold's A: split(v * gamma), fp32 products as its loop forms them
            const float u[4] = {v[0] * g2[0], v[1] * g2[1], v[2] * g2[2], v[3] * g2[3]};
            store_split(ro2, m, u, true);
          }
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
        if constexpr (O_SPLIT) {
          // the consumer GEMM's pre-split A: hi = fp16(v), lo = fp16(v - hi) (v - hi exact in fp32:
          // bitwise the parts that GEMM's split would form from the fp32 v). Lanes ec and ec ^ 1
          // hold the two halves of one 8-column group: they swap (DPP quad_perm [1,0,3,2]), then
          // the even lane stores the group's 16 B of hi parts and the odd lane its 16 B of lo parts.
          store_split(ro, m, v, false);
        } else
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

// ---- launch helpers shared by gemm.hip and gemm_presplit.hip (defined in gemm.hip)
int pick_cfg(int M, int N, int esz);   // tile configuration for a 16-bit GEMM shape
int num_cus();
bool deep_small();                      // 4-slot ring for grids of at most one tile per CU
bool gemm_t96();                        // PREC fp32s: 96-row tiles for better-filled one-round grids
int pp_grid(int nwg, int cus);          // ping-pong launches: blocks per grid
unsigned long long* gemm_stamp_buf();   // CLIPK_GEMM_STAMP diagnostic buffer (or null)
// the same, for this launch only when it passes CLIPK_GEMM_STAMP_EPI / CLIPK_GEMM_STAMP_MINM
unsigned long long* gemm_stamp_for(int epi, int M);
int gemm_skew();                        // CLIPK_GEMM_SKEW (us), 0 when unset
// PREC fp32s launches with pre-split operands (gemm_presplit.hip): spf = the kernel's SPF bits,
// epi the internal epilogue id, lnm the LayerNorm mode; CLIPK_EINVAL for a combination not built
int presplit_launch(bool w16, int spf, int epi, int lnm, const GemmArgs& g, hipStream_t st);

// BM x 256 ping-pong launch when built in and the shape has >= 2 K tiles (the 256-row forms
// with an fp32 residual / aux operand would spill: they keep the 2-slot loop)
template <typename T, typename TO, typename TX, int EPI, int BM, int LNM = 0, int SPF = 0>
static bool try_pp(const GemmArgs& g, int nwg, hipStream_t st) {
  constexpr bool ext32 = (EPI == CLIPK_EPI_BIAS_RES || EPI == CLIPK_EPI_DQGELU || EPI == EPI_DMUL) && sizeof(TX) == 4;
  if constexpr (CLIPK_GEMM_PP && (sizeof(T) == 2 || is_split_v<T>) && !(BM == 256 && ext32)) {
    if (g.K * (int)sizeof(T) < 2 * GEMM_ROWB) return false;
    hipLaunchKernelGGL((gemm_nt_kernel<T, TO, TX, EPI, BM, 256, 2, 4, true, GEMM_ROWB, 2, false, true, LNM, SPF>),
                       dim3(pp_grid(nwg, num_cus())), dim3(512), 0, st, g);
    return true;
  }
  return false;
}

// PREC fp32s (CLIPK_F32S) launches: fp32 out / residual / aux. Large M (where the 16-bit policy
// picks the 192- or 256-row tiles): the ping-pong loop on 192x256 tiles (256-row ones spill at
// 256 VGPRs with the split's temporaries); otherwise 128x128 tiles (a 4-slot ring when the grid
// is at most one tile per CU).
// (Until the split8 hazard above was found, CLIPK_F32S16 ran the 2-MFMA kernel on the ping-pong
// tiles only: on the 2- / 4-slot loop it measured not bit-identical. With the compiler-visible
// split there it is bitwise the 3-MFMA kernel on every tile path, profiles/r05w16/hazard.txt.)
template <int EPI, int LNM = 0, typename TS = f32s, int SPF = 0>
static int launch_gemm_split(const GemmArgs& g, hipStream_t st) {
  const int cus = num_cus();
  const_cast<GemmArgs&>(g).stamp = gemm_stamp_for(EPI, g.M);
  const_cast<GemmArgs&>(g).skew = gemm_skew();
  const int cfg = pick_cfg(g.M, g.N, 2);
  if (cfg == 7) {  // small M (the ViT): 64x128 tiles, twice the 128x128 grid
    const int nwg = ((g.M + 63) / 64) * (g.N / 128);
    if (nwg <= cus && deep_small())
      hipLaunchKernelGGL((gemm_nt_kernel<TS, float, float, EPI, 64, 128, 2, 2, false, GEMM_ROWB, 4, false, false, LNM, SPF>), dim3(nwg),
                         dim3(256), 0, st, g);
    else
      hipLaunchKernelGGL((gemm_nt_kernel<TS, float, float, EPI, 64, 128, 2, 2, false, GEMM_ROWB, 2, false, false, LNM, SPF>), dim3(nwg),
                         dim3(256), 0, st, g);
    CLIPK_CHECK_LAUNCH();
    return CLIPK_OK;
  }
  if (cfg == 1 || cfg == 6) {
    if (try_pp<TS, float, float, EPI, 192, LNM, SPF>(g, ((g.M + 191) / 192) * (g.N / 256), st)) {
      CLIPK_CHECK_LAUNCH();
      return CLIPK_OK;
    }
  }
  const int nwg = ((g.M + 127) / 128) * (g.N / 128);
  // 96-row tiles where they still fit one round of CUs and fill more of it (the batch-1 text
  // encoder's N = 512 GEMMs at 5.9k rows: 188 -> 248 blocks on 256 CUs); knob CLIPK_GEMM_T96
  const int nwg96 = ((g.M + 95) / 96) * (g.N / 128);
  if (nwg < cus && nwg96 <= cus && nwg96 > nwg && deep_small() && gemm_t96())
    hipLaunchKernelGGL((gemm_nt_kernel<TS, float, float, EPI, 96, 128, 2, 2, false, GEMM_ROWB, 4, false, false, LNM, SPF>), dim3(nwg96),
                       dim3(256), 0, st, g);
  else if (nwg <= cus && deep_small())
    hipLaunchKernelGGL((gemm_nt_kernel<TS, float, float, EPI, 128, 128, 2, 2, false, GEMM_ROWB, 4, false, false, LNM, SPF>), dim3(nwg),
                       dim3(256), 0, st, g);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<TS, float, float, EPI, 128, 128, 2, 2, false, GEMM_ROWB, 2, false, false, LNM, SPF>), dim3(nwg),
                       dim3(256), 0, st, g);
  CLIPK_CHECK_LAUNCH();
  return CLIPK_OK;
}

}  // namespace clipk
