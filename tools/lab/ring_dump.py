"""Outputs of the 128x128 GEMM tiles at row counts where the 4-slot ring runs (one tile per CU),
for a same-inputs comparison across CLIPK_GEMM_DEEP=1 (ring) / 0 (2-slot) processes:
    python tools/lab/ring_dump.py OUT.pt ; python tools/lab/ring_dump.py --cmp A.pt B.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    if sys.argv[1] == "--cmp":
        a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
        for k in a:
            x, y = a[k].double(), b[k].double()
            d = ((x - y).abs().max() / y.abs().max()).item()
            print(f"{k}: {int((a[k] != b[k]).sum())} of {x.numel()} differ, rel {d:.2e}", flush=True)
        return
    from fsp_amd import ops, _native as N
    dev = torch.device("cuda")
    out = {}
    for M in (4096, 4600, 8000):
        g = torch.Generator(device="cpu").manual_seed(M)
        a = torch.randn(M, 2048, generator=g).to(dev)
        b = (torch.randn(512, 2048, generator=g) / 2048 ** 0.5).half().float().to(dev)
        bp = ops.split_pack(b)
        out[f"f32s_{M}"] = ops.gemm(a, bp, N.EPI_NONE).cpu()
        out[f"f32h_{M}"] = ops.gemm(a, bp, N.EPI_NONE, w16=True).cpu()
        out[f"f16_{M}"] = ops.gemm(a.half(), b.half(), N.EPI_NONE, torch.float16).cpu()
        out[f"bf16_{M}"] = ops.gemm(a.bfloat16(), b.bfloat16(), N.EPI_NONE, torch.bfloat16).cpu()
    torch.save(out, sys.argv[1])
    print("saved", sys.argv[1], flush=True)


if __name__ == "__main__":
    main()
