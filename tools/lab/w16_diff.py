"""CLIPK_F32S16 vs CLIPK_F32S on an fp16-valued weight across row counts (tile paths): count of
differing outputs and max relative difference. python tools/lab/w16_diff.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fsp_amd import ops, _native as N  # noqa: E402

dev = torch.device("cuda")
for (Nn, K) in ((512, 2048), (2048, 512)):
    for M in (300, 1000, 2000, 4096, 4600, 8000, 20000, 47160):
        g = torch.Generator(device="cpu").manual_seed(M)
        a = torch.randn(M, K, generator=g).to(dev)
        b = (torch.randn(Nn, K, generator=g) / K ** 0.5).half().float().to(dev)
        bp = ops.split_pack(b)
        o3 = ops.gemm(a, bp, N.EPI_NONE)
        o2 = ops.gemm(a, bp, N.EPI_NONE, w16=True)
        ref = a.double() @ b.double().t()
        d = ((o2.double() - o3.double()).abs().max() / o3.double().abs().max()).item()
        e2 = ((o2.double() - ref).abs().max() / ref.abs().max()).item()
        e3 = ((o3.double() - ref).abs().max() / ref.abs().max()).item()
        bad = (o2 != o3).nonzero()
        rows = sorted(set((bad[:, 0] // 64).tolist()))[:6] if len(bad) else []
        cols = sorted(set((bad[:, 1] // 64).tolist()))[:8] if len(bad) else []
        print(f"N {Nn} K {K} M {M}: {len(bad)} differ, rel {d:.2e}, err2 {e2:.2e} err3 {e3:.2e} "
              f"row64 {rows} col64 {cols}", flush=True)
