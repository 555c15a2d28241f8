"""Per-launch time of the N = 512 input-grad GEMM shape (fp16, EPI_NONE) at row counts that give
whole rounds of 256x256 or 192x256 tiles, HIP events, A rotated through HBM (cold).

    python tools/tile_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd import ops, _native as N  # noqa: E402


def timed(fn, it=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    dev = torch.device("cuda")
    lib = N.load()
    K, Nn = 2048, 512
    B = (torch.randn(Nn, K, device=dev) / K ** 0.5).half()
    pool = [torch.randn(47160, K, device=dev).half() for _ in range(4)]  # > 512 MB: streams from HBM
    for cfg, M in [(1, 32768), (1, 47160), (6, 47160), (6, 49152), (1, 29184), (6, 21888), (1, 14592)]:
        lib.clipk_gemm_set_config(cfg)
        k = [0]

        def fn():
            a = pool[k[0] % len(pool)][:M]
            k[0] += 1
            ops.gemm(a, B, N.EPI_NONE, torch.float16)
        us = timed(fn)
        rows = 256 if cfg == 1 else 192
        tiles = ((M + rows - 1) // rows) * (Nn // 256)
        print(f"cfg {cfg} ({rows}x256)  M {M:6d}  tiles {tiles:4d}  {us:7.1f} us  "
              f"{2.0 * M * Nn * K / us / 1e6:7.1f} TF/s  {us / max(1, -(-tiles // 256)):6.1f} us/round", flush=True)
    lib.clipk_gemm_set_config(-1)


if __name__ == "__main__":
    main()
