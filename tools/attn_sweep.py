"""Shared-prefix attention fwd / bwd at the bench shape (CoCoOp ViT-B/16 text, G = 8 images,
C = 1000 classes, P = 5), timed with HIP events on the launch stream; one process per knob
setting (the CLIPK_PREFIX_* knobs are read once per process).

    python tools/attn_sweep.py            # sweep (spawns one child per setting)
    python tools/attn_sweep.py --one      # time the current environment's setting
    python tools/attn_sweep.py --anyl     # the fp32 any-L forward (attn_fwd_f32): ViT-B/16
                                          # L = 197 (100 images) and plain text L = 77 (causal)
"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(iters=30):
    import torch
    from fsp_amd import ops, _native as N
    from fsp_amd.trainers.prompt_base import attention_tiles
    dev = torch.device("cuda")
    G, C, P, H = 8, 1000, 5, 8
    W = H * 64
    g = torch.Generator().manual_seed(0)
    qlen = torch.randint(5, 8, (C,), generator=g)
    off = P + torch.cat([torch.zeros(1, dtype=torch.long), qlen.cumsum(0)[:-1]])
    R = int(P + qlen.sum())
    tl, rf = attention_tiles(off.numpy(), qlen.numpy(), R)
    tiles = torch.from_numpy(tl.reshape(-1).copy()).to(dev)
    row_first = torch.from_numpy(rf).to(dev)
    nt = tiles.numel() // 2
    # SWEEP_DTYPE=fp32: the fp32 kernels (PREC fp32 / fp32s), which also read the forward output
    f32 = os.environ.get("SWEEP_DTYPE", "fp16") == "fp32"
    dt, did, esz = (torch.float32, N.F32, 4) if f32 else (torch.float16, N.F16, 2)
    qkv = (torch.randn(G * R, 3 * W, device=dev) * 0.5).to(dt)
    dout = (torch.randn(G * R, W, device=dev) * 0.5).to(dt)
    dq = torch.empty(G * R, 3 * W, device=dev, dtype=dt)
    nb = N.load().clipk_attention_prefix_ws_bytes(G, nt, H)
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    # clean-cache flush: READ 1 GiB (a write flush would leave the 256-MB Infinity Cache full
    # of dirty lines that the timed kernel then pays to evict)
    flush = torch.ones(1 << 28, dtype=torch.float32, device=dev)
    mode = os.environ.get("SWEEP_CACHE", "clean")
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    o, lse = ops.attention_prefix(qkv, G, P, R, tiles, row_first, H, lse=True)

    def bwd():
        N.call("clipk_attention_prefix_bwd", did, did, G, P, R, nt, p(tiles), p(row_first), H, p(qkv),
               3 * W, p(o), W, p(dout), W, p(lse), p(dq), 3 * W, p(ws), nb, sp)

    def fwd():
        N.call("clipk_attention_prefix_fwd", did, G, P, R, nt, p(tiles), p(row_first), H, p(qkv), 3 * W,
               p(o), W, p(lse), sp)

    rows = G * R
    res = {"rows": rows, "tiles_per_group": nt}
    for name, fn, by in (("fwd", fwd, rows * W * 4 * esz + 4 * rows * H),
                         ("bwd", bwd, rows * W * (9 if f32 else 8) * esz + 4 * rows * H)):
        ts = []
        for i in range(iters + 3):
            if mode == "clean":
                flush.max()
            elif mode == "dirty":
                flush.zero_()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            fn()
            b.record(st)
            torch.cuda.synchronize()
            if i >= 3:
                ts.append(a.elapsed_time(b))
        ts.sort()
        ms = ts[len(ts) // 2]
        res[name] = {"us": round(ms * 1e3, 1), "GBs": round(by / ms / 1e6, 1), "hbm_frac": round(by / ms / 1e6 / 8000, 3)}
    print(json.dumps(res), flush=True)


SWEEP = [
    {"CLIPK_PREFIX_LDS": "0"},
    {"CLIPK_PREFIX_LDS": "0", "CLIPK_PREFIX_WPB": "8"},
    {},
    {"CLIPK_PREFIX_LDS_WPB": "4"},
    {"CLIPK_PREFIX_LDS": "3", "CLIPK_PREFIX_LDS_WPB": "4"},
    {"CLIPK_PREFIX_LDS_WPB": "4", "CLIPK_PREFIX_FWD_CHUNK": "4", "CLIPK_PREFIX_BWD_CHUNK": "8"},
    {"CLIPK_PREFIX_LDS": "0", "SWEEP_CACHE": "warm"},
    {"CLIPK_PREFIX_LDS_WPB": "4", "SWEEP_CACHE": "warm"},
    {"CLIPK_PREFIX_LDS": "0", "SWEEP_CACHE": "dirty"},
    {"CLIPK_PREFIX_LDS_WPB": "4", "SWEEP_CACHE": "dirty"},
]


def anyl(iters=30):
    import torch
    from fsp_amd import _native as N
    dev = torch.device("cuda")
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    flush = torch.ones(1 << 28, dtype=torch.float32, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    res = {}
    for name, nseq, L, H, causal in (("vit_L197", 100, 197, 12, 0), ("text_L77", 1000, 77, 8, 1)):
        W = H * 64
        qkv = torch.randn(nseq * L, 3 * W, device=dev) * 0.5
        o = torch.empty(nseq * L, W, device=dev)
        lse = torch.empty(nseq * L, H, device=dev)
        ts = []
        for i in range(iters + 3):
            flush.max()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            N.call("clipk_attention_fwd", N.F32, nseq, L, H, causal, p(qkv), 3 * W, p(o), W, p(lse), sp)
            b.record(st)
            torch.cuda.synchronize()
            if i >= 3:
                ts.append(a.elapsed_time(b))
        ts.sort()
        res[name] = {"us": round(ts[len(ts) // 2] * 1e3, 1)}
    print(json.dumps(res), flush=True)


def main():
    if "--anyl" in sys.argv:
        anyl()
        return
    if "--one" in sys.argv:
        one()
        return
    for env in SWEEP:
        e = dict(os.environ, **env)
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--one"], env=e, capture_output=True,
                             text=True, timeout=300)
        line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-400:]
        print(json.dumps(env), line, flush=True)
        if out.returncode != 0:
            sys.exit(out.returncode)


if __name__ == "__main__":
    main()
