// Loader / consumer ring GEMM lab (not part of libclipk.so): C[M,N] = A[M,K] . B[N,K]^T, fp16 in,
// fp32 accumulate, fp16 out, on the step's text GEMM shapes -- to measure the structure before it
// moves into csrc/gemm.hip. Driven by tools/lab/ring_lab.py (ctypes + torch).
//
// ring<NS, MODE>: persistent blocks of 8 waves, one per CU, tile 192 x 256, K staged 32 deep
// (64-B rows) into an NS-slot LDS ring:
//  * waves 4..7 (one per SIMD) are LOADERS: each step they issue the LDS-DMA (buffer_load ... lds)
//    of K step g + D (D = NS - 1) and wait (counted vmcnt) until step g + 2 has landed;
//  * waves 0..3 (one per SIMD) are CONSUMERS, each owning a 192 x 64 column slice of the tile
//    (12 x 4 MFMA 16x16x32 sub-tiles, 192 accumulators): per step they read the 4 B fragments of
//    step g + 1 (prefetch), stream the 12 A fragments of step g one ahead of their 4 MFMAs each,
//    and keep the step-g B fragments in registers;
//  * one s_barrier per step for all 8 waves publishes step g + 2 and retires the reads of step g.
// So the MFMA wave never issues a global load, and the LDS-DMA issue cost lands on a wave with
// nothing else to do. MODE bits: 1 = no MFMA (loads + LDS reads + barriers only), 2 = no loads
// after the prologue.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mma(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                0, 0);
}

#define RAW_BARRIER()                  \
  do {                                 \
    __builtin_amdgcn_sched_barrier(0); \
    __builtin_amdgcn_s_barrier();      \
    __builtin_amdgcn_sched_barrier(0); \
  } while (0)

template <int N>
__device__ __forceinline__ void vm_wait() {
  if constexpr (N <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  const unsigned n = bytes <= 0 ? 0u : bytes >= 0x7fffffffLL ? 0x7fffffffu : (unsigned)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)n, 0x00020000);
}

constexpr int BM = 192, BN = 256, ROWB = 64;            // tile, staged bytes per row (32 halfs)
constexpr int OPA = BM * ROWB, SLOT = (BM + BN) * ROWB;  // 12 KB + 16 KB
constexpr int TM = BM / 16, TN = BN / 4 / 16;            // consumer sub-tiles: 12 x 4
// LDS image of a 64-B row: 16-B chunk c of row r stored at chunk c ^ swz(r). For the ds_read_b128
// lane groups of the 16x16x32 fragment reads (lane = row r (0..15) + 16 * chunk) this puts every
// group's 16 lanes on 16 distinct 16-B slots of the 256-B bank row (conflict-free).
__device__ __forceinline__ int swz(int r) { return ((r >> 3) & 1) << 1; }
constexpr int GPS = SLOT / 1024;                         // LDS-DMA instructions per slot: 28
constexpr int LPW = GPS / 4;                             // per loader wave: 7 (A: 3, B: 4)
static_assert(GPS % 4 == 0 && OPA / 1024 == 12 && (BN * ROWB) / 1024 == 16, "slot split");

// ABLK: A in the K-blocked layout [M / BM][K / 32][BM][32] (each ring slot's A part one contiguous
// 12 KB, each LDS-DMA instruction 1 KB contiguous) instead of row-major [M][K] (8 or 16 rows of
// 64-128 B per instruction, rows K * 2 bytes apart): whether the load path is limited by the
// scattered row pieces rather than by bytes.
template <int NS, int MODE, int WARM, bool ABLK = false>
__global__ __launch_bounds__(512, 1) void ring(const f16* __restrict__ A, const f16* __restrict__ B, f16* C, int M,
                                               int N, int K) {
  constexpr int D = NS - 1;
  // + a junk area for the L2-warming loads (LDS-DMA of 4 B per lane, never read)
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT + 4 * 256];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool loader = w >= 4;
  const int ntn = N / BN, ntm = (M + BM - 1) / BM, ntiles = ntm * ntn;
  // XCD-aware bijective split of the tile list: XCD group x owns [t_beg, t_end), walked by the
  // blocks of that group with stride gridDim.x / 8 (tiles sharing an A panel on one XCD)
  const int bid = blockIdx.x, xcd = bid & 7, q = ntiles >> 3, r = ntiles & 7;
  const int t_beg = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int t_end = t_beg + (xcd < r ? q + 1 : q);
  const int t_step = gridDim.x >> 3;
  const int t0 = t_beg + (bid >> 3);
  if (t0 >= t_end) return;  // block-uniform
  const int nk = K * 2 / ROWB;
  const int ntile_mine = (t_end - t0 + t_step - 1) / t_step;
  const int nsteps = ntile_mine * nk;  // global step g over this block's tiles

  if (loader) {
    // loader wave lw stages 1-KiB units lw*LPW .. +LPW of each slot: units 0..11 = A (16 rows
    // each), 12..27 = B. Lane: row lane / 4 of the unit, 16-B chunk (lane % 4) ^ swz(row).
    const int lw = w - 4;
    int poff[LPW];
    bool isa[LPW];
    int urow[LPW];
#pragma unroll
    for (int i = 0; i < LPW; ++i) {
      const int u = lw * LPW + i;
      isa[i] = u < 12;
      const int row = (isa[i] ? u : u - 12) * 16 + lane / 4;
      urow[i] = row;
      const int c = (lane % 4) ^ swz(row);
      poff[i] = (ABLK && isa[i] ? row * ROWB : row * K * 2) + c * 16;
    }
    auto issue = [&](int g) {
      if (g >= nsteps) return;
      const int ti = g / nk, kt = g - ti * nk;
      const int tile = t0 + ti * t_step;
      const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
      const __amdgpu_buffer_rsrc_t ra = rsrc(A + (size_t)m0 * K, (long long)(M - m0) * K * 2);
      const __amdgpu_buffer_rsrc_t rb = rsrc(B + (size_t)n0 * K, (long long)BN * K * 2);
      char* base = smem + (g % NS) * SLOT;
#pragma unroll
      for (int i = 0; i < LPW; ++i) {
        const int u = lw * LPW + i;
        // blocked A: the panel's K step kt is the contiguous BM x 64 B block kt
        const int soff = (ABLK && isa[i]) ? kt * BM * ROWB : kt * ROWB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(isa[i] ? ra : rb,
                                                 (__attribute__((address_space(3))) void*)(base + u * 1024), 16,
                                                 poff[i], soff, 0, 0);
      }
      (void)urow;
    };
    // WARM > 0: one 4-B LDS-DMA per lane into the junk area touches the 128-B line of A row
    // (lw * 48 + lane % 48) at K step g + WARM, so the step's LDS-DMA WARM - D steps later finds
    // it in L2 (the HBM latency is paid outside the LDS ring's in-flight budget)
    const int wrow = lw * 48 + lane % 48;
    auto warm = [&](int g) {
      if constexpr (WARM > 0) {
        if (g >= nsteps) g = nsteps - 1;  // keep the op count per step constant
        const int ti = g / nk, kt = g - ti * nk;
        const int tile = t0 + ti * t_step;
        const int m0 = (tile / ntn) * BM;
        const __amdgpu_buffer_rsrc_t ra = rsrc(A + (size_t)m0 * K, (long long)(M - m0) * K * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(smem + NS * SLOT + lw * 256),
                                                 4, wrow * K * 2, kt * ROWB, 0, 0);
      }
    };
    constexpr int OPS = LPW + (WARM > 0 ? 1 : 0);  // vm ops per step per loader wave
    if constexpr (WARM > 0)
      for (int g = 0; g < WARM; ++g) warm(g);
    for (int g = 0; g < D; ++g) {
      issue(g);
      warm(g + WARM);
    }
    vm_wait<(D - 2) * OPS>();  // steps 0 and 1 landed
    RAW_BARRIER();
    for (int g = 0; g < nsteps; ++g) {
      if (!(MODE & 2)) {
        issue(g + D);
        warm(g + D + WARM);
      }
      // step g + 2 landed (D - 2 younger steps stay in flight); past the end: everything
      if (g + D < nsteps) vm_wait<(D - 2) * OPS>();
      else vm_wait<0>();
      RAW_BARRIER();
    }
    return;
  }

  // ---- consumers: wave w owns columns [64 w, 64 w + 64) of the tile
  const int fr = lane & 15, fq = lane >> 4;
  const int swzr = swz(fr);  // sub-tile rows are multiples of 16: row & 15 = fr
  const int cofs = ((fq ^ swzr) << 4);
  const int arow0 = fr * ROWB + cofs;                      // + i * 16 * ROWB
  const int brow0 = OPA + (w * 64 + fr) * ROWB + cofs;     // + j * 16 * ROWB
  auto afrag = [&](int slot, int i) {
    return *reinterpret_cast<const u32x4*>(smem + slot * SLOT + arow0 + i * 16 * ROWB);
  };
  auto bfrag = [&](int slot, int j) {
    return *reinterpret_cast<const u32x4*>(smem + slot * SLOT + brow0 + j * 16 * ROWB);
  };
  RAW_BARRIER();  // steps 0, 1 published
  u32x4 bc[TN], bn[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bc[j] = bfrag(0, j);
  int g = 0;
  for (int ti = 0; ti < ntile_mine; ++ti) {
    const int tile = t0 + ti * t_step;
    const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // one K step: B of step g + 1 prefetched into the other register set, A of step g streamed
    // one sub-tile ahead of its 4 MFMAs; PAR (compile time) says which set holds step g's B
    auto kstep = [&](auto PAR) {
      constexpr int par = decltype(PAR)::value;
      u32x4* cur = par ? bn : bc;
      u32x4* nxt = par ? bc : bn;
      const int s = g % NS, sn = (g + 1) % NS;
#pragma unroll
      for (int j = 0; j < TN; ++j) nxt[j] = bfrag(sn, j);  // (past the end: a harmless re-read)
      // A fragments AHEAD sub-tiles ahead of their MFMAs (compile-time indices: ~AHEAD+1 live)
      constexpr int AHEAD = 3;
      u32x4 af[TM];
#pragma unroll
      for (int i = 0; i < AHEAD; ++i) af[i] = afrag(s, i);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (i + AHEAD < TM) af[i + AHEAD] = afrag(s, i + AHEAD);
        if constexpr (!(MODE & 1)) {
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma(cur[j], af[i], acc[i][j]);
        } else {
          asm volatile("" ::"v"(af[i]));
        }
      }
      if constexpr (MODE & 1) {
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(cur[j]));
      }
      ++g;
      RAW_BARRIER();
    };
    // nk is even (checked by the launcher): every tile starts with the B set bc current
    for (int kt = 0; kt < nk; kt += 2) {
      kstep(std::integral_constant<int, 0>());
      kstep(std::integral_constant<int, 1>());
    }
    // epilogue (direct stores; the lab measures the K loop)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + i * 16 + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + w * 64 + j * 16 + fq * 4;
        f16x4 v = {(f16)acc[i][j][0], (f16)acc[i][j][1], (f16)acc[i][j][2], (f16)acc[i][j][3]};
        *reinterpret_cast<f16x4*>(C + (size_t)m * N + n) = v;
      }
    }
  }
}

template <int NS, int MODE, int WARM, bool ABLK = false>
static int launch(const void* A, const void* B, void* C, int M, int N, int K, int grid, hipStream_t st) {
  if (N % BN || (K * 2) % (2 * ROWB)) return -2;  // an even number of 32-deep K steps
  if (ABLK && M % BM) return -4;
  hipLaunchKernelGGL((ring<NS, MODE, WARM, ABLK>), dim3(grid), dim3(512), 0, st, (const f16*)A, (const f16*)B, (f16*)C, M, N,
                     K);
  return (int)hipGetLastError();
}

extern "C" int ring_gemm(int ns, int warm, int mode, const void* A, const void* B, void* C, int M, int N, int K, int grid,
                         void* stream) {
  hipStream_t st = (hipStream_t)stream;
  grid = (grid / 8) * 8;
  if (grid <= 0) return -3;
#define V(NSV, WV)                                                                      \
  if (ns == NSV && warm == WV) {                                                        \
    if (mode == 0) return launch<NSV, 0, WV>(A, B, C, M, N, K, grid, st);               \
    if (mode == 1) return launch<NSV, 1, WV>(A, B, C, M, N, K, grid, st);               \
    if (mode == 2) return launch<NSV, 2, WV>(A, B, C, M, N, K, grid, st);               \
  }
  V(4, 0)
  V(5, 0)
  V(5, 4)
  V(5, 8)
  V(4, 8)
#undef V
  if (ns == 5 && warm == 100) {  // blocked A (the caller passes A in the [M/192][K/32][192][32] layout)
    if (mode == 0) return launch<5, 0, 0, true>(A, B, C, M, N, K, grid, st);
    if (mode == 1) return launch<5, 1, 0, true>(A, B, C, M, N, K, grid, st);
    if (mode == 2) return launch<5, 2, 0, true>(A, B, C, M, N, K, grid, st);
  }
  return -1;
}
