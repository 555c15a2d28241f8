"""Batch-1 text GEMM shapes (M = 5,895 packed rows at C = 1,000; N = 512 input-grad GEMMs,
EPI_NONE, fp16): the tile-grid launch (ops.gemm) against split-K (ops.gemm_splitk: fp32 slice
partials + the fixed-order finish pass) at 2 / 3 / 4 slices and the library's own choice.
A rotated over 4 buffers; HIP events, best of 3 rounds of 20 launches.
    python tools/lab/b1_splitk.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fsp_amd import ops, _native as N  # noqa: E402


def timeit(fn, iters=20, rounds=3):
    for i in range(3):
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
    return best * 1e3


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for M in (5895, 2950, 1475):
        for n, k, name in ((512, 2048, "fc_dx"), (512, 1536, "qkv_dx"), (512, 512, "out_dx")):
            As = [(torch.randn(M, k, device=dev, generator=g) * 0.5).half() for _ in range(4)]
            B = (torch.randn(n, k, device=dev, generator=g) * 0.5).half()
            ref = As[0].float() @ B.float().t()
            t0 = timeit(lambda i: ops.gemm(As[i % 4], B, N.EPI_NONE, torch.float16))
            line = f"M {M:5d} {name:7s} K {k:4d}: grid {t0:6.1f} us"
            for sp in (2, 3, 4, 0):
                o = ops.gemm_splitk(As[0], B, N.EPI_NONE, torch.float16, splits=sp)
                torch.cuda.synchronize()
                err = ((o.float() - ref).abs().max() / ref.abs().max()).item()
                t = timeit(lambda i: ops.gemm_splitk(As[i % 4], B, N.EPI_NONE, torch.float16, splits=sp))
                auto = N.load().clipk_gemm_auto_splits(N.F16, M, n, k) if sp == 0 else sp
                line += f" | splitK {sp if sp else f'auto={auto}'} {t:6.1f} us" + (" WRONG" if err > 1e-2 else "")
            print(line, flush=True)
            del As, B, ref


if __name__ == "__main__":
    main()
