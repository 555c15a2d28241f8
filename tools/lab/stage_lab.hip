// Staging-path lab (not part of libclipk.so): how fast one CU can move GEMM operand tiles from
// L2 / HBM into LDS by LDS-DMA (buffer_load_dwordx4 ... lds, what the production ping-pong loop
// issues) against register staging (buffer_load_dwordx4 into VGPRs, then ds_write_b128, what
// hipBLASLt's kernels do), with no MFMA work: the same 192 + 256 row panels of 128 B per K step
// as the 192x256 GEMM tile, rows K * 2 bytes apart, DEPTH K steps in flight, all 8 waves
// issuing. Driven by tools/lab/stage_lab.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  const unsigned n = bytes <= 0 ? 0u : bytes >= 0x7fffffffLL ? 0x7fffffffu : (unsigned)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)n, 0x00020000);
}

constexpr int BM = 192, BN = 256, ROWB = 128, STAGE = (BM + BN) * ROWB;  // 56 KiB per K step
constexpr int UNITS = STAGE / 1024;  // 1-KiB pieces (8 rows x 128 B) per stage: 56, 7 per wave

// MODE 0: LDS-DMA; MODE 1: registers + ds_write_b128; MODE 2: registers only (no LDS write)
// BLK: the operands pre-blocked, each K step's 192-row A panel and 256-row B panel one
// contiguous run (as a packed layout would hold them) instead of 128-B row pieces 2K bytes apart.
// PF > 0 (LDS-DMA only): one 4-B load per 128-B line of the A panel PF K steps ahead, issued
// after the next stage's DMA and left in flight (an L2 warm-up of the first-touch activations)
// AA / AB: cache-policy bits of the A / B LDS-DMA loads (1 sc0, 2 nt, 16 sc1)
template <int MODE, int DEPTH, bool BLK = false, int PF = 0, int AA = 0, int AB = 0>
__global__ __launch_bounds__(512, 1) void stage_kernel(const char* __restrict__ A, const char* __restrict__ B, int M,
                                                       int K, int ntiles, int* sink) {
  __shared__ __attribute__((aligned(16))) char smem[MODE == 2 ? 1024 : DEPTH * STAGE];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nk = K * 2 / ROWB;
  const int ntn = 2;  // N = 512: two 256-column tiles
  u32x4 reg[DEPTH][7];
  u32x4 acc = {0u, 0u, 0u, 0u};
  unsigned pf = 0;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
    const __amdgpu_buffer_rsrc_t ra = rsrc(A + (size_t)m0 * K * 2, (long long)(M - m0) * K * 2);
    const __amdgpu_buffer_rsrc_t rb = rsrc(B + (size_t)n0 * K * 2, (long long)BN * K * 2);
    auto issue = [&](int kt, int slot) {
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const int u = w * 7 + i;           // unit: A 0..23, B 24..55
        const bool ua = u < BM / 8;
        const int row = (ua ? u : u - BM / 8) * 8 + lane / 8;
        const int off = BLK ? row * ROWB + (lane % 8) * 16 : row * K * 2 + (lane % 8) * 16;
        const int koff = BLK ? kt * (ua ? BM : BN) * ROWB : kt * ROWB;
        if constexpr (MODE == 0) {
          if (ua)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(smem + slot * STAGE + u * 1024),
                                                     16, off, koff, 0, AA);
          else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (__attribute__((address_space(3))) void*)(smem + slot * STAGE + u * 1024),
                                                     16, off, koff, 0, AB);
        } else {
          reg[slot][i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ua ? ra : rb, off + koff, 0, 0));
        }
      }
    };
    auto land = [&](int slot) {  // registers -> LDS (MODE 1) or a use that keeps the loads (MODE 2)
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        if constexpr (MODE == 1)
          *reinterpret_cast<u32x4*>(smem + slot * STAGE + (w * 7 + i) * 1024 + lane * 16) = reg[slot][i];
        else if constexpr (MODE == 2)
          acc ^= reg[slot][i];
      }
    };
#pragma unroll
    for (int d = 0; d < DEPTH - 1; ++d) issue(d, d);
    for (int kt = 0; kt < nk; ++kt) {
      const int slot = kt % DEPTH;
      if (kt + DEPTH - 1 < nk) {
        // slot (kt + DEPTH - 1) % DEPTH was consumed at step kt - 1 (barrier below)
        switch ((kt + DEPTH - 1) % DEPTH) {
          case 0: issue(kt + DEPTH - 1, 0); break;
          case 1: if (DEPTH > 1) issue(kt + DEPTH - 1, 1 % DEPTH); break;
          default: if (DEPTH > 2) issue(kt + DEPTH - 1, 2 % DEPTH); break;
        }
        if constexpr (PF > 0) {
          // 192 A rows per K step: lanes of waves 0..2 touch one line each
          if (w < 3) {
            const int kp = kt + PF < nk ? kt + PF : nk - 1;
            pf ^= __builtin_amdgcn_raw_buffer_load_b32(ra, (w * 64 + lane) * K * 2 + kp * ROWB, 0, 0);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          } else {
            asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
          }
        } else if constexpr (DEPTH == 3) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      switch (slot) {
        case 0: land(0); break;
        case 1: if (DEPTH > 1) land(1 % DEPTH); break;
        default: if (DEPTH > 2) land(2 % DEPTH); break;
      }
      __syncthreads();
      if constexpr (MODE != 2) acc ^= *reinterpret_cast<const u32x4*>(smem + (kt % DEPTH) * STAGE + threadIdx.x * 16);
      __syncthreads();
    }
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3] ^ pf) == 0x9e3779b9u) sink[0] = 1;  // keep the loads live
}

extern "C" int stage_lab(int mode, int depth, const void* A, const void* B, int M, int K, int grid, void* sink,
                         void* stream) {
  if (mode >= 10) {  // pre-blocked operands (mode - 10)
    const int ntiles = ((M + BM - 1) / BM) * 2;
    hipStream_t st = (hipStream_t)stream;
    if (depth != 2) return -1;
    if (mode >= 30) {
#define P(AAV, ABV) hipLaunchKernelGGL((stage_kernel<0, 2, false, 0, AAV, ABV>), dim3(grid), dim3(512), 0, st, (const char*)A, (const char*)B, M, K, ntiles, (int*)sink)
      if (mode == 30) P(2, 0); else if (mode == 31) P(1, 0); else if (mode == 32) P(2, 2); else if (mode == 33) P(16, 0);
      else if (mode == 34) P(0, 2); else P(3, 0);
#undef P
      return (int)hipGetLastError();
    }
    if (mode == 12)
      hipLaunchKernelGGL((stage_kernel<0, 2, false, 2>), dim3(grid), dim3(512), 0, st, (const char*)A, (const char*)B, M, K, ntiles, (int*)sink);
    else if (mode == 13)
      hipLaunchKernelGGL((stage_kernel<0, 2, false, 4>), dim3(grid), dim3(512), 0, st, (const char*)A, (const char*)B, M, K, ntiles, (int*)sink);
    else if (mode == 14)
      hipLaunchKernelGGL((stage_kernel<0, 2, false, 8>), dim3(grid), dim3(512), 0, st, (const char*)A, (const char*)B, M, K, ntiles, (int*)sink);
    else if (mode == 10)
      hipLaunchKernelGGL((stage_kernel<0, 2, true>), dim3(grid), dim3(512), 0, st, (const char*)A, (const char*)B, M, K, ntiles, (int*)sink);
    else
      hipLaunchKernelGGL((stage_kernel<1, 2, true>), dim3(grid), dim3(512), 0, st, (const char*)A, (const char*)B, M, K, ntiles, (int*)sink);
    return (int)hipGetLastError();
  }
  const int ntiles = ((M + BM - 1) / BM) * 2;
  hipStream_t st = (hipStream_t)stream;
#define L(MO, DE) hipLaunchKernelGGL((stage_kernel<MO, DE>), dim3(grid), dim3(512), 0, st, (const char*)A, (const char*)B, M, K, ntiles, (int*)sink)
  if (depth == 2) {
    if (mode == 0) L(0, 2); else if (mode == 1) L(1, 2); else L(2, 2);
  } else if (mode == 2) {
    L(2, 3);
  } else {
    return -1;  // three 56-KiB stages exceed the 160 KiB of LDS
  }
#undef L
  return (int)hipGetLastError();
}
