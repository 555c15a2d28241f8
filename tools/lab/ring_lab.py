"""Drive tools/lab/libringlab.so (ring_lab.hip: loader / consumer ring GEMM) on the step's text
GEMM shapes (M = 47,160) against the production GEMM (ops.gemm) and hipBLASLt, A rotated over
> 600 MB of buffers (HBM-resident as in the step). HIP events, best of 3 rounds of 12 launches.
    python tools/lab/ring_lab.py [ns list] [mode list]"""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from fsp_amd import ops, _native as N  # noqa: E402

MODES = {0: "full", 1: "no-MFMA", 2: "no-loads", 3: "no-MFMA no-loads"}


def timeit(fn, iters=12, warm=3, rounds=3):
    for i in range(warm):
        fn(i)
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for i in range(iters):
            fn(i)
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / iters)
    return best


def main():
    nss = [tuple(int(x) for x in v.split("w")) for v in (sys.argv[1] if len(sys.argv) > 1 else "4w0,5w0").split(",")]
    modes = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,1,2").split(",")]
    M = int(os.environ.get("RING_M", 47232))  # 246 x 192 (the blocked-A variant needs M % 192 == 0)
    grid = int(os.environ.get("RING_GRID", 256))
    lib = ctypes.CDLL(os.path.join(HERE, "libringlab.so"))
    lib.ring_gemm.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 4 + \
        [ctypes.c_void_p]
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for n, k in ((512, 2048), (512, 1536), (512, 512), (2048, 512), (1536, 512)):
        nbuf = max(2, -(-600_000_000 // (M * k * 2)))
        As = [(torch.randn(M, k, device=dev, generator=g) * 0.5).half() for _ in range(nbuf)]
        B = (torch.randn(n, k, device=dev, generator=g) * 0.5).half()
        C = torch.empty(M, n, device=dev, dtype=torch.float16)
        fl = 2.0 * M * n * k
        ref = (As[0].float() @ B.float().t())
        # blocked copies of A for the ABLK variant (ns 5, warm 100): [M/192][K/32][192][32]
        Ab = [a.view(M // 192, 192, k // 32, 32).permute(0, 2, 1, 3).contiguous() if any(w == 100 for _, w in nss)
              else None for a in As]
        ms = timeit(lambda i: ops.gemm(As[i % nbuf], B, N.EPI_NONE, torch.float16, out=C))
        print(f"N{n} K{k}: ours(prod auto) {ms*1e3:7.1f} us {fl/ms/1e9:7.1f} TF/s", flush=True)
        ms = timeit(lambda i: torch.matmul(As[i % nbuf], B.t(), out=C))
        print(f"N{n} K{k}: hipBLASLt       {ms*1e3:7.1f} us {fl/ms/1e9:7.1f} TF/s", flush=True)
        for ns, wm in nss:
            for md in modes:
                C.zero_()
                AA = Ab if wm == 100 else As
                rc = lib.ring_gemm(ns, wm, md, AA[0].data_ptr(), B.data_ptr(), C.data_ptr(), M, n, k, grid, st())
                if rc:
                    print(f"  ring ns{ns}w{wm} mode {md}: rc {rc}")
                    continue
                err = ""
                if md == 0:
                    torch.cuda.synchronize()
                    e = ((C.float() - ref).abs().max() / ref.abs().max()).item()
                    err = f" relerr {e:.1e}" + ("  <-- WRONG" if e > 1e-2 else "")
                ms = timeit(lambda i: lib.ring_gemm(ns, wm, md, AA[i % nbuf].data_ptr(), B.data_ptr(), C.data_ptr(), M,
                                                    n, k, grid, st()))
                print(f"  ring ns{ns}w{wm} {MODES[md]:17s} {ms*1e3:7.1f} us {fl/ms/1e9:7.1f} TF/s{err}", flush=True)
        del As, Ab, B, C, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
