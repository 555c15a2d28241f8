"""hipBLASLt (torch.matmul) on the step's N=512 / N=2048 shapes, for a rocprofv3 kernel trace."""
import torch
dev = torch.device("cuda")
M = 47160
for n, k in ((512, 2048), (512, 1536), (512, 512), (2048, 512), (1536, 512)):
    a = (torch.randn(M, k, device=dev) * 0.5).half()
    b = (torch.randn(n, k, device=dev) * 0.5).half()
    for _ in range(5):
        torch.matmul(a, b.t())
    torch.cuda.synchronize()
