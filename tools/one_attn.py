"""Run the shared-prefix attention fwd+bwd at the bench shape N times (rocprofv3 PMC passes).
Usage: one_attn.py [iters]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd import ops, _native as N  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda")
G, C, P, H = 8, 1000, 5, 8
W = H * 64
qlen = torch.full((C,), 6, dtype=torch.long)
qlen[:100] = 5
off = P + torch.cat([torch.zeros(1, dtype=torch.long), qlen.cumsum(0)[:-1]])
R = int(P + qlen.sum())
from fsp_amd.trainers.prompt_base import attention_tiles  # noqa: E402
tl, rf = attention_tiles(off.numpy(), qlen.numpy(), R)
tiles = torch.from_numpy(tl.reshape(-1).copy()).to(dev)
row_first = torch.from_numpy(rf).to(dev)
nt = tiles.numel() // 2
qkv = (torch.randn(G * R, 3 * W, device=dev) * 0.5).to(torch.float16)
dout = (torch.randn(G * R, W, device=dev) * 0.5).to(torch.bfloat16)
dq = torch.empty(G * R, 3 * W, device=dev, dtype=torch.bfloat16)
nb = N.load().clipk_attention_prefix_ws_bytes(G, tiles.numel() // 2, H)
ws = torch.empty(nb, dtype=torch.uint8, device=dev)
p = lambda t: ctypes.c_void_p(t.data_ptr())
for _ in range(it):
    o, lse = ops.attention_prefix(qkv, G, P, R, tiles, row_first, H, lse=True)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    N.call("clipk_attention_prefix_bwd", N.F16, N.BF16, G, P, R, tiles.numel() // 2, p(tiles), p(row_first), H, p(qkv), 3 * W, p(o), W, p(dout),
           W, p(lse), p(dq), 3 * W, p(ws), nb, st)
torch.cuda.synchronize()
print("done", it)
