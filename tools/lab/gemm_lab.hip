// GEMM structure lab (not part of libclipk.so): C[M,N] = A[M,K] . B[N,K]^T, fp16 in, fp32
// accumulate, fp16 out, to measure K-loop designs on the step's text GEMM shapes before
// moving one into csrc/gemm.hip. Driven by tools/lab/gemm_lab.py (ctypes + torch).
//
// lab<BM, BN, WM, WN, ROWB, S, MODE>: BM x BN block tile, WM x WN waves (each TM x TN MFMA
// 16x16x32 sub-tiles, operands swapped so a lane holds 4 consecutive output columns), K staged
// ROWB bytes per row (64 halfs = 128 B or 32 halfs = 64 B) into an S-slot LDS ring by
// global_load_lds_dwordx4 with a source-side XOR swizzle (conflict-free for the ds_read_b128
// lane groups).
//  S == 2: the classic loop -- issue stage s+1, read + MMA stage s, vmcnt(0), barrier.
//  S >= 3: software-pipelined -- the fragments of MFMA window v+1 are read while window v's
//          MFMAs run (A fragments re-read right after their last use, B double-buffered), stage
//          s+S-1 is issued at the top of step s into the slot whose readers all passed the
//          barrier ending step s-1, and the end-of-step counted vmcnt retires only stage s+2
//          (S-3 stages stay in flight across the raw s_barrier).
// MODE bits (experiments): 1 = no MFMA, 2 = no global loads after the prologue.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

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

template <int BM, int BN, int WM, int WN, int ROWB, int S, int MODE>
__global__ __launch_bounds__(WM* WN * 64, 1) void lab(const f16* __restrict__ A, const f16* __restrict__ B,
                                                      f16* C, int M, int N, int K) {
  constexpr int NW = WM * WN, TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int OPA = BM * ROWB, STAGE = (BM + BN) * ROWB;
  constexpr int RPI = 1024 / ROWB, CPR = ROWB / 16, KW = ROWB / 64;  // rows / glds, chunks / row, windows / step
  constexpr int IA = BM / RPI / NW, IB = BN / RPI / NW, PER = IA + IB;
  static_assert(IA >= 1 && IB >= 1 && BM % (RPI * NW) == 0 && BN % (RPI * NW) == 0, "tile / wave");
  __shared__ __attribute__((aligned(16))) char smem[S * STAGE];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w / WN, wn = w % WN;

  // XCD-aware bijective tile order (tiles sharing an A row panel on one XCD)
  const int ntn = N / BN, ntm = (M + BM - 1) / BM, nwg = ntm * ntn;
  const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int nk = K * 2 / ROWB;  // K steps
  auto swz = [](int rr) { return ROWB == 128 ? ((rr >> 1) & 7) : (((rr >> 3) & 1) << 1); };

  const char* srcA[IA];
  const char* srcB[IB];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int row = (w * IA + i) * RPI + lane / CPR;
    int ga = m0 + row;
    ga = ga < M ? ga : M - 1;
    srcA[i] = (const char*)(A + (size_t)ga * K) + ((lane % CPR) ^ swz(row)) * 16;
  }
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int row = (w * IB + i) * RPI + lane / CPR;
    srcB[i] = (const char*)(B + (size_t)(n0 + row) * K) + ((lane % CPR) ^ swz(row)) * 16;
  }
  auto stage = [&](int s) {
    char* base = smem + (s % S) * STAGE;
    const size_t koff = (size_t)s * ROWB;
#pragma unroll
    for (int i = 0; i < IA; ++i) glds16(srcA[i] + koff, base + (w * IA + i) * 1024);
#pragma unroll
    for (int i = 0; i < IB; ++i) glds16(srcB[i] + koff, base + OPA + (w * IB + i) * 1024);
  };

  const int fr = lane & 15, fq = lane >> 4, sw = swz(fr);
  // fragment of MFMA window v (K step v / KW, 64-B window v % KW of its staged rows)
  auto a_frag = [&](int v, int i) {
    const int s = v / KW, kk = v % KW;
    return *reinterpret_cast<const u32x4*>(smem + (s % S) * STAGE + (wm * (BM / WM) + i * 16 + fr) * ROWB +
                                           (((kk * 4 + fq) ^ sw) << 4));
  };
  auto b_frag = [&](int v, int j) {
    const int s = v / KW, kk = v % KW;
    return *reinterpret_cast<const u32x4*>(smem + (s % S) * STAGE + OPA + (wn * (BN / WN) + j * 16 + fr) * ROWB +
                                           (((kk * 4 + fq) ^ sw) << 4));
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if constexpr (S == 2) {
    stage(0);
    vm_wait<0>();
    __syncthreads();
    for (int s = 0; s < nk; ++s) {
      if (!(MODE & 2) && s + 1 < nk) stage(s + 1);
#pragma unroll
      for (int kk = 0; kk < KW; ++kk) {
        u32x4 a[TM], b[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = b_frag(s * KW + kk, j);
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = a_frag(s * KW + kk, i);
        if constexpr (!(MODE & 1)) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = mma(b[j], a[i], acc[i][j]);
        } else {
#pragma unroll
          for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(a[i]));
#pragma unroll
          for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(b[j]));
        }
      }
      vm_wait<0>();
      __syncthreads();
    }
  } else {
    // prologue: stages 0..S-2 in flight; stage 0 retired and published, window 0 read;
    // stage 1 retired and published before step 0
    for (int s = 0; s < S - 1; ++s)
      if (s < nk) stage(s);
    vm_wait<(S - 2) * PER>();
    RAW_BARRIER();
    u32x4 fa[TM], fb[2][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[i] = a_frag(0, i);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[0][j] = b_frag(0, j);
    if (S == 3 || nk < 2) vm_wait<0>();
    else vm_wait<(S - 3) * PER>();
    RAW_BARRIER();
    const int nwin = nk * KW;
    // one MFMA window v with B register set CUR; reads window v+1's fragments behind it
    auto window = [&](int v, auto CURT) {
      constexpr int cur = decltype(CURT)::value;
      // always read (the last window re-reads itself): a conditional read becomes a
      // per-register select that keeps both values live
      const int vn = v + 1 < nwin ? v + 1 : v;
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[cur ^ 1][j] = b_frag(vn, j);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if constexpr (!(MODE & 1)) {
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma(fb[cur][j], fa[i], acc[i][j]);
        } else {
          asm volatile("" ::"v"(fa[i]));
        }
        fa[i] = a_frag(vn, i);
      }
    };
    auto step_end = [&](int s) {
      // retire stage s+2 (first read during step s+1); stages s+3.. stay in flight
      if (s + 2 < nk) {
        if (s + S - 1 < nk) vm_wait<(S - 3) * PER>();
        else vm_wait<0>();
      }
      RAW_BARRIER();
    };
    auto kstep = [&](int s, auto CURT) {
      if (!(MODE & 2) && s + S - 1 < nk) stage(s + S - 1);
      if constexpr (KW == 2) {
        window(2 * s, std::integral_constant<int, 0>());
        window(2 * s + 1, std::integral_constant<int, 1>());
      } else {
        window(s, CURT);
      }
      step_end(s);
    };
    // step pairs: the B register set alternates with the window, a compile-time index
    for (int s = 0; s < nk; s += 2) {
      kstep(s, std::integral_constant<int, 0>());
      if (s + 1 < nk) kstep(s + 1, std::integral_constant<int, 1>());
    }
  }

  // epilogue (direct stores; not what the lab measures)
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * (BM / WM) + i * 16 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * (BN / WN) + j * 16 + fq * 4;
      f16x4 v = {(f16)acc[i][j][0], (f16)acc[i][j][1], (f16)acc[i][j][2], (f16)acc[i][j][3]};
      *reinterpret_cast<f16x4*>(C + (size_t)m * N + n) = v;
    }
  }
}

template <int BM, int BN, int WM, int WN, int ROWB, int S, int MODE>
static int launch(const void* A, const void* B, void* C, int M, int N, int K, hipStream_t st) {
  if (N % BN || (K * 2) % ROWB) return -2;
  const int nwg = ((M + BM - 1) / BM) * (N / BN);
  hipLaunchKernelGGL((lab<BM, BN, WM, WN, ROWB, S, MODE>), dim3(nwg), dim3(WM * WN * 64), 0, st, (const f16*)A,
                     (const f16*)B, (f16*)C, M, N, K);
  return (int)hipGetLastError();
}


// labreg<BM, BN, WM, WN, MODE>: register-staged loads with 2 K steps of lead (Tensile's
// PGR2 scheme): at step s the global loads of stage s+1 (issued two steps earlier) are
// waited for and written to LDS slot (s+1)&1, the loads of stage s+3 are issued into the
// register set just freed, then the MFMAs of stage s run on slot s&1; one barrier per step.
// K staged 64 halfs (128-B rows); LDS XOR swizzle applied on the ds_write side.
template <int BM, int BN, int WM, int WN, int MODE>
__global__ __launch_bounds__(WM* WN * 64, 1) void labreg(const f16* __restrict__ A, const f16* __restrict__ B,
                                                         f16* C, int M, int N, int K) {
  constexpr int NT = WM * WN * 64, TM = BM / WM / 16, TN = BN / WN / 16, ROWB = 128;
  constexpr int OPA = BM * ROWB, STAGE = (BM + BN) * ROWB;
  constexpr int CA = BM * 8 / NT, CB = BN * 8 / NT;  // 16-B chunks per thread per stage
  static_assert(BM * 8 % NT == 0 && BN * 8 % NT == 0, "chunks / thread");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w / WN, wn = w % WN;
  const int ntn = N / BN, ntm = (M + BM - 1) / BM, nwg = ntm * ntn;
  const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int nk = K / 64;
  auto swz = [](int rr) { return (rr >> 1) & 7; };
  const char* ga[CA];
  const char* gb[CB];
  int la[CA], lb[CB];
#pragma unroll
  for (int i = 0; i < CA; ++i) {
    const int c = t + NT * i, row = c >> 3, ch = c & 7;
    int g = m0 + row;
    g = g < M ? g : M - 1;
    ga[i] = (const char*)(A + (size_t)g * K) + ch * 16;
    la[i] = row * ROWB + ((ch ^ swz(row)) << 4);
  }
#pragma unroll
  for (int i = 0; i < CB; ++i) {
    const int c = t + NT * i, row = c >> 3, ch = c & 7;
    gb[i] = (const char*)(B + (size_t)(n0 + row) * K) + ch * 16;
    lb[i] = OPA + row * ROWB + ((ch ^ swz(row)) << 4);
  }
  u32x4 ra[2][CA], rb[2][CB];
  auto gload = [&](int s, auto SETT) {
    constexpr int set = decltype(SETT)::value;
    const size_t ko = (size_t)(s < nk ? s : nk - 1) * ROWB;
#pragma unroll
    for (int i = 0; i < CA; ++i) ra[set][i] = *reinterpret_cast<const u32x4*>(ga[i] + ko);
#pragma unroll
    for (int i = 0; i < CB; ++i) rb[set][i] = *reinterpret_cast<const u32x4*>(gb[i] + ko);
  };
  auto lwrite = [&](int slot, auto SETT) {
    constexpr int set = decltype(SETT)::value;
    char* base = smem + slot * STAGE;
#pragma unroll
    for (int i = 0; i < CA; ++i) *reinterpret_cast<u32x4*>(base + la[i]) = ra[set][i];
#pragma unroll
    for (int i = 0; i < CB; ++i) *reinterpret_cast<u32x4*>(base + lb[i]) = rb[set][i];
  };
  const int fr = lane & 15, fq = lane >> 4, sw = swz(fr);
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int slot) {
    const char* As = smem + slot * STAGE + (wm * (BM / WM) + fr) * ROWB;
    const char* Bs = smem + slot * STAGE + OPA + (wn * (BN / WN) + fr) * ROWB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int p = ((kk * 4 + fq) ^ sw) << 4;
      u32x4 a[TM], b[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = *reinterpret_cast<const u32x4*>(Bs + j * 16 * ROWB + p);
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = *reinterpret_cast<const u32x4*>(As + i * 16 * ROWB + p);
      if constexpr (!(MODE & 1)) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma(b[j], a[i], acc[i][j]);
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(a[i]));
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(b[j]));
      }
    }
  };
  // prologue: stage 0 -> LDS slot 0; stages 1, 2 in flight in register sets 1, 0
  gload(0, std::integral_constant<int, 0>());
  lwrite(0, std::integral_constant<int, 0>());
  gload(1, std::integral_constant<int, 1>());
  gload(2, std::integral_constant<int, 0>());
  __syncthreads();
  auto kstep = [&](int s, auto SETT) {  // SETT: register set holding stage s+1
    constexpr int set = decltype(SETT)::value;
    // branch-free body (a conditional here makes the compiler drain every load at the merge):
    // past the last stage the writes land in the idle slot and the loads re-read stage nk-1
    lwrite((s + 1) & 1, SETT);                   // waits for stage s+1's loads only
    if constexpr (!(MODE & 2)) gload(s + 3, SETT);  // refill the freed set
    compute(s & 1);
    __syncthreads();
  };
  for (int s = 0; s < nk; s += 2) {
    kstep(s, std::integral_constant<int, 1>());
    if (s + 1 < nk) kstep(s + 1, std::integral_constant<int, 0>());
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * (BM / WM) + i * 16 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * (BN / WN) + j * 16 + fq * 4;
      f16x4 v = {(f16)acc[i][j][0], (f16)acc[i][j][1], (f16)acc[i][j][2], (f16)acc[i][j][3]};
      *reinterpret_cast<f16x4*>(C + (size_t)m * N + n) = v;
    }
  }
}

template <int BM, int BN, int WM, int WN, int MODE>
static int launch_reg(const void* A, const void* B, void* C, int M, int N, int K, hipStream_t st) {
  if (N % BN || K % 64) return -2;
  const int nwg = ((M + BM - 1) / BM) * (N / BN);
  hipLaunchKernelGGL((labreg<BM, BN, WM, WN, MODE>), dim3(nwg), dim3(WM * WN * 64), 0, st, (const f16*)A,
                     (const f16*)B, (f16*)C, M, N, K);
  return (int)hipGetLastError();
}

// variant ids (tools/lab/gemm_lab.py names them)
extern "C" int lab_gemm(int variant, int mode, const void* A, const void* B, void* C, int M, int N, int K,
                        void* stream) {
  hipStream_t st = (hipStream_t)stream;
#define V(ID, BM, BN, WM, WN, ROWB, S)                                              \
  if (variant == ID) {                                                               \
    if (mode == 0) return launch<BM, BN, WM, WN, ROWB, S, 0>(A, B, C, M, N, K, st); \
    if (mode == 1) return launch<BM, BN, WM, WN, ROWB, S, 1>(A, B, C, M, N, K, st); \
    if (mode == 2) return launch<BM, BN, WM, WN, ROWB, S, 2>(A, B, C, M, N, K, st); \
    if (mode == 3) return launch<BM, BN, WM, WN, ROWB, S, 3>(A, B, C, M, N, K, st); \
  }
  V(0, 256, 256, 2, 4, 128, 2)  // the production structure (cfg 1, non-persistent)
  V(1, 192, 256, 2, 4, 128, 2)  // production cfg 6
  V(2, 256, 256, 2, 4, 64, 4)   // 8 waves, BK 32, 4-slot ring, pipelined fragments
  V(3, 256, 256, 2, 4, 64, 5)   // 5-slot ring
  V(5, 256, 256, 2, 4, 64, 3)   // 3-slot ring (no stage in flight across the barrier)
  V(6, 256, 256, 2, 2, 128, 2)  // 4 waves (one per SIMD), 128x128 per wave, classic 2-slot
  // full-N tiles for the N = 512 GEMMs (A row panel staged once per K step, not once per
  // 256-column tile): 192 x 512, BK 32 (64-B rows), 45 KB per stage
  V(10, 192, 512, 1, 4, 64, 3)  // 4 waves of 192x128 (384 accumulators), 3-slot pipelined
  V(11, 192, 512, 1, 4, 64, 2)  // same, classic 2-slot
  V(13, 192, 512, 2, 2, 64, 3)  // 4 waves of 96x256 (384 accumulators), 3-slot pipelined
#undef V
#define R(ID, BM, BN, WM, WN)                                                     \
  if (variant == ID) {                                                             \
    if (mode == 0) return launch_reg<BM, BN, WM, WN, 0>(A, B, C, M, N, K, st);    \
    if (mode == 1) return launch_reg<BM, BN, WM, WN, 1>(A, B, C, M, N, K, st);    \
    if (mode == 2) return launch_reg<BM, BN, WM, WN, 2>(A, B, C, M, N, K, st);    \
  }
  R(8, 192, 256, 2, 4)  // register-staged, 2 steps of lead
  R(9, 256, 256, 2, 4)
#undef R
  return -1;
}
