"""A/B of the LayerNorm-fold GEMM epilogues against the plain ones on the headline text shapes
(M = 47,160 packed rows, W = 512), isolated launches, HIP events:
consumers (qkv N 1536 EPI_BIAS, c_fc N 2048 EPI_BIAS_QGELU with h) and producers (out_proj
K 512, c_proj K 2048: EPI_BIAS_RES with / without the statistics partials), plus the merge."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd import ops, _native as N  # noqa: E402
from fsp_amd.clip import model as M  # noqa: E402
from tools.kbench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    dt = torch.float16
    Mr, W = int(os.environ.get("AB_ROWS", 47160)), 512
    g = torch.Generator(device="cpu").manual_seed(0)
    x = (torch.randn(Mr, W, generator=g) + torch.randn(Mr, 1, generator=g)).to(dev, dt)
    gamma = (1 + 0.05 * torch.randn(W, generator=g)).to(dev)
    beta = (0.02 * torch.randn(W, generator=g)).to(dev)
    xg = x.double().reshape(Mr, W // 64, 64)
    st_x = torch.stack([xg.sum(-1), ((xg - xg.mean(-1, keepdim=True)) ** 2).sum(-1)], -1).float().contiguous()
    _, _, rnb = ops.ln_stats_merge(st_x, W)
    for Nn, epi, nm in ((1536, N.EPI_BIAS, "qkv"), (2048, N.EPI_BIAS_QGELU, "c_fc")):
        w = (torch.randn(Nn, W, generator=g) / math.sqrt(W)).to(dev)
        b = (0.02 * torch.randn(Nn, generator=g)).to(dev)
        wp, s, c = M.ln_fold_weights(w, b, gamma, beta, dt, dev)
        wq = w.to(dt)
        q2 = epi == N.EPI_BIAS_QGELU
        t_plain = timeit(lambda: ops.gemm(x, wq, epi, dt, bias=b, want_out2=q2), iters=20)
        t_fold = timeit(lambda: ops.gemm_ln(x, wp, epi, c, colsum=s, rnb=rnb, want_out2=q2), iters=20)
        fl = 2.0 * Mr * Nn * W
        print(f"{nm:8s} plain {t_plain * 1e3:7.1f} us ({fl / t_plain / 1e9:6.1f} TF/s)   fold {t_fold * 1e3:7.1f} us "
              f"({fl / t_fold / 1e9:6.1f} TF/s)")
    for K, nm in ((512, "out_proj"), (2048, "c_proj")):
        a = torch.randn(Mr, K, generator=g).to(dev, dt)
        w = (torch.randn(W, K, generator=g) / math.sqrt(K)).to(dev, dt)
        b = (0.02 * torch.randn(W, generator=g)).to(dev)
        st = torch.empty(Mr, W // 64, 2, device=dev)
        t_plain = timeit(lambda: ops.gemm(a, w, N.EPI_BIAS_RES, dt, bias=b, res=x), iters=20)
        t_st = timeit(lambda: ops.gemm_ln(a, w, N.EPI_BIAS_RES, b, st, res=x), iters=20)
        t_m = timeit(lambda: ops.ln_stats_merge(st, W), iters=20)
        t_ln = timeit(lambda: ops.layernorm(x, gamma, beta, out_dtype=dt, stats=True), iters=20)
        fl = 2.0 * Mr * W * K
        print(f"{nm:8s} plain {t_plain * 1e3:7.1f} us ({fl / t_plain / 1e9:6.1f} TF/s)   stats {t_st * 1e3:7.1f} us  "
              f"merge {t_m * 1e3:5.1f} us  (LayerNorm pass {t_ln * 1e3:5.1f} us)")


if __name__ == "__main__":
    main()
