"""Every text-encoder GEMM of the CoCoOp train step (M = 8 images x 5895 packed rows) under
each GEMM tile configuration in KB_CFGS (default: automatic choice and the 8-phase cfg 7).
Prints per-launch time (HIP events over 20 launches, median of 3) and TFLOP/s."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd import ops, _native as N  # noqa: E402


def timeit(fn, iters=20, warm=3, reps=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / iters)
    return sorted(out)[len(out) // 2]


def main():
    dev = torch.device("cuda")
    M = int(os.environ.get("KB_M", 47160))
    W = 512
    f16, bf = torch.float16, torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s, dt=f16: (torch.randn(*s, device=dev, generator=g) * 0.5).to(dt)  # noqa: E731
    x, xb = rnd(M, W), rnd(M, W, dt=bf)
    h4, h4b = rnd(M, 4 * W), rnd(M, 4 * W, dt=bf)
    bias3, bias1, bias4 = (torch.randn(n, device=dev) for n in (3 * W, W, 4 * W))
    wqkv, wo, w1, w2 = rnd(3 * W, W), rnd(W, W), rnd(4 * W, W), rnd(W, 4 * W)
    wqkvT, woT, w1T, w2T = rnd(W, 3 * W, dt=bf), rnd(W, W, dt=bf), rnd(W, 4 * W, dt=bf), rnd(4 * W, W, dt=bf)
    q3b = rnd(M, 3 * W, dt=bf)
    res16 = rnd(M, W)
    shapes = [
        ("fwd qkv    N1536 K512  bias", 3 * W, W, lambda: ops.gemm(x, wqkv, N.EPI_BIAS, f16, bias=bias3)),
        ("fwd out    N512  K512  res16", W, W, lambda: ops.gemm(x, wo, N.EPI_BIAS_RES, f16, bias=bias1, res=res16)),
        ("fwd fc1    N2048 K512  qgelu+h", 4 * W, W,
         lambda: ops.gemm(x, w1, N.EPI_BIAS_QGELU, f16, bias=bias4, want_out2=True)),
        ("fwd fc2    N512  K2048 res16", W, 4 * W, lambda: ops.gemm(h4, w2, N.EPI_BIAS_RES, f16, bias=bias1, res=res16)),
        ("bwd fc2^T  N2048 K512  dgelu", 4 * W, W, lambda: ops.gemm(xb, w2T, N.EPI_DQGELU, bf, aux=h4)),
        ("bwd fc1^T  N512  K2048 bf16", W, 4 * W, lambda: ops.gemm(h4b, w1T, N.EPI_NONE, bf)),
        ("bwd qkv^T  N512  K1536 bf16", W, 3 * W, lambda: ops.gemm(q3b, wqkvT, N.EPI_NONE, bf)),
        ("bwd out^T  N512  K512  bf16", W, W, lambda: ops.gemm(xb, woT, N.EPI_NONE, bf)),
    ]
    cfgs = [int(c) for c in os.environ.get("KB_CFGS", "-1,7").split(",")]
    tot = {c: 0.0 for c in cfgs}
    for name, n, k, fn in shapes:
        line = f"{name:32s}"
        for c in cfgs:
            N.load().clipk_gemm_set_config(c)
            ms = timeit(fn)
            mult = 12 if "fc" in name or "qkv" in name or "out" in name else 1
            tot[c] += ms * mult
            line += f" | cfg{c:>2d} {ms*1e3:7.1f} us {2*M*n*k/ms/1e9:6.0f} TF/s"
        print(line, flush=True)
    N.load().clipk_gemm_set_config(-1)
    print("x12 layers: " + "  ".join(f"cfg{c} {t:.2f} ms" for c, t in tot.items()))


if __name__ == "__main__":
    main()
