"""ViT small-M GEMM forms (HIP events, isolated launches): tile configurations forced by
clipk_gemm_set_config (0 = 128x128, 7 = 64x128) against split-K (auto slices), on the ViT
shapes at 8 images (B/16: M 1,576; L/14@336: M 4,616)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd import ops, _native as N  # noqa: E402
from tools.kbench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    dt = torch.float16
    lib = N.load()
    shapes = [("B16 qkv", 1576, 2304, 768, N.EPI_BIAS), ("B16 out", 1576, 768, 768, N.EPI_BIAS_RES),
              ("B16 fc", 1576, 3072, 768, N.EPI_BIAS_QGELU), ("B16 proj", 1576, 768, 3072, N.EPI_BIAS_RES),
              ("L336 qkv", 4616, 3072, 1024, N.EPI_BIAS), ("L336 out", 4616, 1024, 1024, N.EPI_BIAS_RES),
              ("L336 fc", 4616, 4096, 1024, N.EPI_BIAS_QGELU), ("L336 proj", 4616, 1024, 4096, N.EPI_BIAS_RES)]
    for nm, M, Nn, K, epi in shapes:
        g = torch.Generator(device="cpu").manual_seed(M + Nn + K)
        a = torch.randn(M, K, generator=g).to(dev, dt)
        b = (torch.randn(Nn, K, generator=g) / math.sqrt(K)).to(dev, dt)
        bias = torch.randn(Nn, generator=g).to(dev)
        od = torch.float32 if epi == N.EPI_BIAS_RES else dt
        res = torch.randn(M, Nn, generator=g).to(dev) if epi == N.EPI_BIAS_RES else None
        kw = dict(bias=bias, res=res)
        t = {}
        for cfg in (-1, 0, 7):
            lib.clipk_gemm_set_config(cfg)
            t[cfg] = timeit(lambda: ops.gemm(a, b, epi, od, **kw), iters=20)
        lib.clipk_gemm_set_config(-1)
        ts = timeit(lambda: ops.gemm_splitk(a, b, epi, od, **kw), iters=20)
        lib.clipk_gemm_set_config(7)
        ts7 = timeit(lambda: ops.gemm_splitk(a, b, epi, od, **kw), iters=20) if epi != N.EPI_BIAS_QGELU else 0
        lib.clipk_gemm_set_config(-1)
        print(f"{nm:10s} M {M:5d} N {Nn:5d} K {K:5d}: auto {t[-1] * 1e3:6.1f}  128x128 {t[0] * 1e3:6.1f}  "
              f"64x128 {t[7] * 1e3:6.1f}  split-K {ts * 1e3:6.1f}  split-K(cfg7 forced) {ts7 * 1e3:6.1f} us")


if __name__ == "__main__":
    main()
