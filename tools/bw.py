"""HBM bandwidth yardsticks on the box: write-only (fill), read-only (sum), copy."""
import torch
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kbench import timeit

dev = torch.device("cuda")
for mb in (193, 386):
    n = mb * 1024 * 1024 // 4
    x = torch.empty(n, device=dev)
    y = torch.empty(n, device=dev)
    ms = timeit(lambda: x.fill_(1.0))
    print(f"fill  {mb} MB  {ms*1e3:8.1f} us  {n*4/ms/1e6:7.1f} GB/s")
    ms = timeit(lambda: y.copy_(x))
    print(f"copy  {mb} MB  {ms*1e3:8.1f} us  {2*n*4/ms/1e6:7.1f} GB/s (r+w)")
    ms = timeit(lambda: x.sum())
    print(f"sum   {mb} MB  {ms*1e3:8.1f} us  {n*4/ms/1e6:7.1f} GB/s")
