"""The step's text GEMM shapes (CoCoOp ViT-B/16, B = 8, C = 1000, shared-prefix packed:
M = 47,160 rows) on our kernel vs hipBLASLt (torch.matmul), in one process, with the A
operand rotated over buffers totalling > 512 MB so that every launch reads A from HBM as
inside the training step (back-to-back launches on one buffer would re-read it from the
256 MB Infinity Cache). HIP events, min over rounds of the mean of `iters` launches.

    python tools/gemm_yardstick.py [M]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd import ops, _native as N  # noqa: E402

W = 512
SHAPES = [  # name, N, K, epi, out dtype, aux/res
    ("qkv_fwd  N1536 K512  BIAS", 3 * W, W, "bias"),
    ("out_fwd  N512  K512  BIAS_RES", W, W, "res"),
    ("fc_fwd   N2048 K512  BIAS", 4 * W, W, "bias"),
    ("proj_fwd N512  K2048 BIAS_RES|AQGELU", W, 4 * W, "res_ag"),
    ("dgelu    N2048 K512  DQGELU", 4 * W, W, "dqgelu"),
    ("fc_dx    N512  K2048 NONE", W, 4 * W, "none"),
    ("out_dx   N512  K512  NONE", W, W, "none"),
    ("qkv_dx   N512  K1536 NONE", W, 3 * W, "none"),
]


def timeit(fn, iters=12, warm=3, rounds=3):
    for i in range(warm):
        fn(i)
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for i in range(iters):
            fn(i)
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / iters)
    return best


VIT = [  # ViT-B/16 layer GEMMs (D = 768) at B = 8 images x 197 tokens
    ("vit qkv  N2304 K768  BIAS", 2304, 768, "bias"),
    ("vit out  N768  K768  BIAS_RES", 768, 768, "res"),
    ("vit fc   N3072 K768  BIAS", 3072, 768, "bias"),
    ("vit proj N768  K3072 BIAS_RES", 768, 3072, "res"),
]


def main():
    global SHAPES
    if "--vit" in sys.argv:
        sys.argv.remove("--vit")
        SHAPES = VIT
        if len(sys.argv) == 1:
            sys.argv.append("1576")
    hot = "--hot" in sys.argv  # one A buffer: re-read from the Infinity Cache / L2
    if hot:
        sys.argv.remove("--hot")
    ref_on = "--no-ref" not in sys.argv
    if not ref_on:
        sys.argv.remove("--no-ref")
    only = None  # --only <name prefix>: one shape (PMC runs)
    if "--only" in sys.argv:
        j = sys.argv.index("--only")
        only = sys.argv[j + 1]
        del sys.argv[j:j + 2]
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 47160
    dev = torch.device("cuda")
    f16 = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: (torch.randn(*s, device=dev, generator=g) * 0.5).to(f16)
    tot_ours = tot_t = 0.0
    for name, n, k, kind in SHAPES:
        if only and not name.startswith(only):
            continue
        nbuf = 1 if hot else max(2, -(-600_000_000 // (M * k * 2)))
        As = [rnd(M, k) for _ in range(nbuf)]
        B = rnd(n, k)
        bias = torch.randn(n, device=dev)
        vit_res = SHAPES is VIT and kind == "res"  # the ViT's residual stream is fp32
        res = torch.randn(M, n, device=dev) if vit_res else rnd(M, n)
        aux = rnd(M, n)
        out = torch.empty(M, n, device=dev, dtype=torch.float32 if vit_res else f16)
        if kind == "none":
            ours = lambda i: ops.gemm(As[i % nbuf], B, N.EPI_NONE, f16, out=out)
        elif kind == "bias":
            ours = lambda i: ops.gemm(As[i % nbuf], B, N.EPI_BIAS, f16, bias=bias, out=out)
        elif kind == "res":
            ours = lambda i: ops.gemm(As[i % nbuf], B, N.EPI_BIAS_RES, out.dtype, bias=bias, res=res, out=out)
        elif kind == "res_ag":
            ours = lambda i: ops.gemm(As[i % nbuf], B, N.EPI_BIAS_RES | N.A_QGELU, f16, bias=bias, res=res,
                                      out=out)
        else:
            ours = lambda i: ops.gemm(As[i % nbuf], B, N.EPI_DQGELU, f16, aux=aux, out=out)
        outr = torch.empty(M, n, device=dev, dtype=f16)
        ref = lambda i: torch.matmul(As[i % nbuf], B.t(), out=outr)
        if SHAPES is VIT and kind in ("bias", "res"):
            sk = N.load().clipk_gemm_auto_splits(N.F16, M, n, k)
            epi = N.EPI_BIAS if kind == "bias" else N.EPI_BIAS_RES
            for s_ in sorted({1, 2, 3, 4, sk}):
                ms_s = timeit(lambda i: ops.gemm_splitk(As[i % nbuf], B, epi, out.dtype, bias=bias,
                                                        res=res if kind == "res" else None, splits=s_))
                print(f"    split-K {s_}{' (auto)' if s_ == sk else ''}: {ms_s*1e3:7.1f} us "
                      f"{2.0*M*n*k/ms_s/1e9:7.1f} TF/s", flush=True)
        ms_o = timeit(ours)
        ms_t = timeit(ref) if ref_on else float("nan")
        fl = 2.0 * M * n * k
        tot_ours += ms_o
        tot_t += ms_t
        print(f"{name:38s} ours {ms_o*1e3:7.1f} us {fl/ms_o/1e9:7.1f} TF/s | hipBLASLt (plain) {ms_t*1e3:7.1f} us "
              f"{fl/ms_t/1e9:7.1f} TF/s", flush=True)
        del As, B, res, aux, out
        torch.cuda.empty_cache()
    print(f"sum ours {tot_ours*1e3:.1f} us | hipBLASLt {tot_t*1e3:.1f} us (hipBLASLt without the fused epilogues)")


if __name__ == "__main__":
    main()
