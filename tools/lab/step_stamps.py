"""Where a persistent GEMM of the real train step spends its time: K steps of the CoCoOp bench
step with in-kernel s_memrealtime stamps on one class of launch (CLIPK_GEMM_STAMP=1 plus the
filter CLIPK_GEMM_STAMP_EPI / CLIPK_GEMM_STAMP_MINM: the buffer keeps the step's last launch of
that class). Per tile: K-loop and epilogue duration, the gap to the next tile, and how aligned
the blocks' epilogues are.
    CLIPK_GEMM_STAMP=1 CLIPK_GEMM_STAMP_EPI=5 CLIPK_GEMM_STAMP_MINM=40000 PREC=fp32s \\
        python tools/lab/step_stamps.py [steps]"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

NB, NT = 2048, 8  # STAMP_BLOCKS, STAMP_TILES of gemm_kernel.h


def report(name):
    from fsp_amd import _native as N
    buf = np.zeros((NB, 4 + 3 * NT), dtype=np.uint64)
    N.check(N.load().clipk_gemm_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes), "stamps")
    used = buf[:, 1] != 0
    b = buf[used].astype(np.int64)
    if not len(b):
        print(f"{name}: no stamped launch", flush=True)
        return
    t0 = b[:, 1].min()
    tiles = b[:, 2:2 + 3 * NT].reshape(len(b), NT, 3) - t0
    ok = tiles[:, :, 2] > 0
    kl = (tiles[:, :, 1] - tiles[:, :, 0])[ok] / 100.0  # us (100 MHz)
    ep = (tiles[:, :, 2] - tiles[:, :, 1])[ok] / 100.0
    gap = (tiles[:, 1:, 0] - tiles[:, :-1, 2])[ok[:, 1:]] / 100.0
    first = tiles[:, 0, 1][ok[:, 0]] / 100.0
    kl0 = (tiles[:, 0, 1] - tiles[:, 0, 0])[ok[:, 0]] / 100.0
    kl1 = (tiles[:, 1:, 1] - tiles[:, 1:, 0])[ok[:, 1:]] / 100.0
    pct = lambda x: f"{np.median(x):6.2f} (p10 {np.percentile(x, 10):.2f} p90 {np.percentile(x, 90):.2f})"
    print(f"{name}: blocks {len(b)}, tiles/block {ok.sum(1).max()}", flush=True)
    print(f"   k-loop/tile {pct(kl)} us; first tile {np.median(kl0):.2f}, later tiles "
          f"{np.median(kl1) if kl1.size else 0:.2f}", flush=True)
    print(f"   epilogue/tile {pct(ep)} us; gap to next tile {np.median(gap) if gap.size else 0:.2f} us", flush=True)
    print(f"   first epilogue start: min {first.min():.2f} p50 {np.median(first):.2f} max {first.max():.2f} us; "
          f"last end {tiles[:, :, 2].max() / 100.0:.2f} us", flush=True)


def main():
    import torch
    import bench
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    prec = os.environ.get("PREC", "fp32s")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr, dm = bench.build_trainer(argparse.Namespace(arch="ViT-B/16", classes=1000), prec, 8, dev, 0)
    t, _ = bench.time_train(tr, dm, steps, 2)
    torch.cuda.synchronize()
    print(f"{prec}: {1000 * t / steps:.3f} ms/step (stamped), EPI {os.environ.get('CLIPK_GEMM_STAMP_EPI')} "
          f"skew {os.environ.get('CLIPK_GEMM_SKEW', '0')}", flush=True)
    report(f"EPI {os.environ.get('CLIPK_GEMM_STAMP_EPI')} M >= {os.environ.get('CLIPK_GEMM_STAMP_MINM', 0)}")


if __name__ == "__main__":
    main()
