"""Diagnostic: where a persistent GEMM launch spends its time, from in-kernel s_memrealtime
marks (run with CLIPK_GEMM_STAMP=1). Per block: k-loop and epilogue duration of each tile,
and how aligned the blocks' epilogues are in time."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd import ops, _native as N  # noqa: E402

NB, NT = 2048, 8


def run(name, fn):
    fn()
    torch.cuda.synchronize()
    fn()
    buf = np.zeros((NB, 4 + 3 * NT), dtype=np.uint64)
    N.check(N.load().clipk_gemm_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes), "stamps")
    used = buf[:, 1] != 0
    b = buf[used].astype(np.int64)
    t0 = b[:, 1].min()
    tiles = b[:, 2:2 + 3 * NT].reshape(len(b), NT, 3) - t0
    clk = (b[:, -2] - b[:, 0]) / ((b[:, -1] - b[:, 1]) / 100.0) / 1e3  # GHz
    ok = tiles[:, :, 2] > 0
    kl = (tiles[:, :, 1] - tiles[:, :, 0])[ok] / 100.0  # us (100 MHz)
    ep = (tiles[:, :, 2] - tiles[:, :, 1])[ok] / 100.0
    gap = (tiles[:, 1:, 0] - tiles[:, :-1, 2])[ok[:, 1:]] / 100.0
    print(f"{name}: blocks {len(b)}  k-loop/tile {np.median(kl):6.2f} us (p10 {np.percentile(kl,10):.2f} "
          f"p90 {np.percentile(kl,90):.2f})  epilogue/tile {np.median(ep):6.2f} us (p10 {np.percentile(ep,10):.2f} "
          f"p90 {np.percentile(ep,90):.2f})  tile gap {np.median(gap) if gap.size else 0:.2f} us  clock {np.median(clk):.2f} GHz")
    # alignment: spread of the first tile's epilogue start across blocks
    e0 = tiles[:, 0, 1] / 100.0
    print(f"   first k-loop end spread: min {e0.min():.2f} p50 {np.median(e0):.2f} max {e0.max():.2f} us; "
          f"last end {tiles[:, :, 2].max() / 100.0:.2f} us")


def main():
    dev = torch.device("cuda")
    M = int(os.environ.get("KB_M", 47160))
    cfg = int(os.environ.get("KB_CFG", "1"))
    N.load().clipk_gemm_set_config(cfg)
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s, dt=torch.float16: (torch.randn(*s, device=dev, generator=g) * 0.5).to(dt)
    a, b = rnd(M, 512), rnd(2048, 512)
    bias = torch.randn(2048, device=dev)
    run("plain f16  N2048 K512", lambda: ops.gemm(a, b, N.EPI_NONE, torch.float16))
    run("plain f32  N2048 K512", lambda: ops.gemm(a, b, N.EPI_NONE, torch.float32))
    run("qgelu+h    N2048 K512", lambda: ops.gemm(a, b, N.EPI_BIAS_QGELU, torch.float16, bias=bias, want_out2=True))
    bb, ab = rnd(2048, 512, dt=torch.bfloat16), rnd(M, 512, dt=torch.bfloat16)
    aux = rnd(M, 2048)
    run("dgelu bf16 N2048 K512", lambda: ops.gemm(ab, bb, N.EPI_DQGELU, torch.bfloat16, aux=aux))
    af, bfc = rnd(M, 2048, dt=torch.bfloat16), rnd(512, 2048, dt=torch.bfloat16)
    run("fcbwd bf16 N512 K2048 ", lambda: ops.gemm(af, bfc, N.EPI_NONE, torch.float32))
    a4, b4 = rnd(M, 2048), rnd(2048, 2048)
    run("plain f16  N2048 K2048", lambda: ops.gemm(a4, b4, N.EPI_NONE, torch.float16))


if __name__ == "__main__":
    main()
