"""Per-launch time of the ViT-B/16 projection GEMMs at B=8 (M = 8 x 197 rows), HIP events."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd import ops, _native as N  # noqa: E402


def t(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


dev = torch.device("cuda")
M, D = 1576, 768
x = torch.randn(M, D, device=dev).half()
h = torch.randn(M, 4 * D, device=dev).half()
wq, wf1 = torch.randn(3 * D, D, device=dev).half() * 0.03, torch.randn(4 * D, D, device=dev).half() * 0.03
wo, wf2 = torch.randn(D, D, device=dev).half() * 0.03, torch.randn(D, 4 * D, device=dev).half() * 0.03
b3, b4, b1 = torch.randn(3 * D, device=dev), torch.randn(4 * D, device=dev), torch.randn(D, device=dev)
res = torch.randn(M, D, device=dev)
print(f"qkv  N2304 K768  {t(lambda: ops.gemm(x, wq, N.EPI_BIAS, torch.float16, bias=b3)):7.1f} us")
print(f"fc1  N3072 K768  {t(lambda: ops.gemm(x, wf1, N.EPI_BIAS_QGELU, torch.float16, bias=b4)):7.1f} us")
print(f"out  N768  K768  {t(lambda: ops.gemm_splitk(x, wo, N.EPI_BIAS_RES, torch.float32, bias=b1, res=res)):7.1f} us (split-K)")
print(f"fc2  N768  K3072 {t(lambda: ops.gemm_splitk(h, wf2, N.EPI_BIAS_RES, torch.float32, bias=b1, res=res)):7.1f} us (split-K)")
print(f"out  N768  K768  {t(lambda: ops.gemm(x, wo, N.EPI_BIAS_RES, torch.float32, bias=b1, res=res)):7.1f} us (no split)")
print(f"fc2  N768  K3072 {t(lambda: ops.gemm(h, wf2, N.EPI_BIAS_RES, torch.float32, bias=b1, res=res)):7.1f} us (no split)")
for s_ in (2, 3, 4, 6):
    print(f"fc2  N768  K3072 {t(lambda: ops.gemm_splitk(h, wf2, N.EPI_BIAS_RES, torch.float32, bias=b1, res=res, splits=s_)):7.1f} us (split {s_})")
for s_ in (2, 3):
    print(f"out  N768  K768  {t(lambda: ops.gemm_splitk(x, wo, N.EPI_BIAS_RES, torch.float32, bias=b1, res=res, splits=s_)):7.1f} us (split {s_})")
