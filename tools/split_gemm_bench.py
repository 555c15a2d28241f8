"""PREC fp32s GEMM shapes of the headline step (M = 47,160 packed text rows) timed alone, HIP
events, A rotated over > 600 MB so it streams from HBM as in the step: the N = 512 input-grad
GEMMs (fc_dx K 2048, qkv_dx K 1536, out_dx K 512), c_proj forward (K 2048, BIAS_RES) and the
N = 2048 / 1536 forward shapes. Weights fp16-valued: mode 2 (compact B, CLIPK_F32S16) and mode 1
(packed B, CLIPK_F32S). CLIPK_LIB selects a library variant (tools/build_variant.sh).

    python tools/split_gemm_bench.py [tag]  -> one line per shape: us per launch, TF/s (fp32 FLOPs)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd import ops, _native as N  # noqa: E402

M = int(os.environ.get("SGB_M", 47160))
SHAPES = [("fc_dx", 512, 2048, N.EPI_NONE), ("qkv_dx", 512, 1536, N.EPI_NONE), ("out_dx", 512, 512, N.EPI_NONE),
          ("proj_fwd", 512, 2048, N.EPI_BIAS_RES), ("fc_fwd", 2048, 512, N.EPI_BIAS), ("qkv_fwd", 1536, 512, N.EPI_BIAS)]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else os.path.basename(os.path.dirname(N.LIB_PATH))
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for name, Nn, K, epi in SHAPES:
        nrot = max(2, int(6e8 // (M * K * 4)) + 1)
        As = [torch.randn(M, K, device=dev, generator=g) for _ in range(nrot)]
        w = (torch.randn(Nn, K, device=dev, generator=g) / K ** 0.5).half().float()
        bp = ops.split_pack(w)
        bh = ops.split_hi16(bp)
        bias = torch.randn(Nn, device=dev, generator=g)
        res = torch.randn(M, Nn, device=dev, generator=g) if epi == N.EPI_BIAS_RES else None
        out = torch.empty(M, Nn, device=dev)
        for mode, b in (("w16", bh), ("mode1", bp)):
            kw = {"bias": bias} if epi != N.EPI_NONE else {}
            if res is not None:
                kw["res"] = res

            def run(i):
                ops.gemm(As[i % nrot], b, epi, out=out, **kw)
            for i in range(5):
                run(i)
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(3):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for i in range(20):
                    run(i)
                e.record()
                torch.cuda.synchronize()
                best = min(best, s.elapsed_time(e) / 20)
            tf = 2.0 * M * Nn * K / (best * 1e-3) / 1e12
            print(f"{tag:10s} {name:9s} {mode:6s} M {M} N {Nn} K {K}: {best * 1000:7.1f} us  {tf:6.1f} TF/s", flush=True)
        del As


if __name__ == "__main__":
    main()
