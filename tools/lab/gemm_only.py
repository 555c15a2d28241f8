"""The production GEMM alone on one text shape (default: fc_dx, M = 47,160 packed rows, N = 512,
K = 2048, EPI_NONE, fp16), A rotated over >600 MB, for PMC passes
(`rocprofv3 --pmc ... -- python3 tools/lab/gemm_only.py`): 20 launches after 3 warm-ups.
    python tools/lab/gemm_only.py [N K]      (BLASLT=1: torch.matmul instead)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fsp_amd import ops, _native as N  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    M = 47160
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    nbuf = max(2, -(-600_000_000 // (M * k * 2)))
    As = [(torch.randn(M, k, device=dev, generator=g) * 0.5).half() for _ in range(nbuf)]
    B = (torch.randn(n, k, device=dev, generator=g) * 0.5).half()
    C = torch.empty(M, n, device=dev, dtype=torch.float16)
    blaslt = os.environ.get("BLASLT")
    for i in range(23):
        if blaslt:  # the same product through hipBLASLt (torch.matmul)
            torch.matmul(As[i % nbuf], B.t(), out=C)
        else:
            ops.gemm(As[i % nbuf], B, N.EPI_NONE, torch.float16, out=C)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
