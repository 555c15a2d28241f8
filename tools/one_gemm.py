"""Run one GEMM shape N times (for rocprofv3 PMC passes). Usage: one_gemm.py <name> [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd import ops, _native as N  # noqa: E402

M, W = int(os.environ.get("KB_M", 47160)), 512
f16, bf = torch.float16, torch.bfloat16
dev = torch.device("cuda")
name = sys.argv[1] if len(sys.argv) > 1 else "dgelu"
it = int(sys.argv[2]) if len(sys.argv) > 2 else 10
a = (torch.randn(M, W, device=dev) * 0.5)
if name == "dgelu":
    A, B = a.to(bf), (torch.randn(4 * W, W, device=dev) * 0.05).to(bf)
    aux = torch.randn(M, 4 * W, device=dev).to(f16)
    fn = lambda: ops.gemm(A, B, N.EPI_DQGELU, bf, aux=aux)
elif name == "plain":
    A, B = a.to(f16), (torch.randn(4 * W, W, device=dev) * 0.05).to(f16)
    fn = lambda: ops.gemm(A, B, N.EPI_NONE, f16)
elif name == "fcbwd":
    A, B = (torch.randn(M, 4 * W, device=dev) * 0.5).to(bf), (torch.randn(W, 4 * W, device=dev) * 0.05).to(bf)
    fn = lambda: ops.gemm(A, B, N.EPI_NONE, torch.float32)
for _ in range(it):
    fn()
torch.cuda.synchronize()
print("done", name, it)
