"""Drive tools/lab/libstagelab.so (stage_lab.hip): staging rate of the 192x256 GEMM tile's
operand panels (N = 512, K = 2048, M = 47,232) into LDS by LDS-DMA vs register staging, no MFMA;
HIP events, best of 3 rounds of 10 launches, A rotated over >600 MB.
    python tools/lab/stage_lab.py"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
NAMES = {0: "LDS-DMA (buffer_load ... lds)", 1: "registers + ds_write_b128", 2: "registers only (no LDS)",
         10: "LDS-DMA, pre-blocked operands", 11: "registers + ds_write, pre-blocked",
         12: "LDS-DMA + A lines warmed 2 ahead", 13: "LDS-DMA + A lines warmed 4 ahead", 14: "LDS-DMA + A lines warmed 8 ahead",
         30: "LDS-DMA, A nt", 31: "LDS-DMA, A sc0", 32: "LDS-DMA, A nt + B nt", 33: "LDS-DMA, A sc1",
         34: "LDS-DMA, B nt", 35: "LDS-DMA, A sc0 nt"}


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libstagelab.so"))
    lib.stage_lab.argtypes = [ctypes.c_int] * 2 + [ctypes.c_void_p] * 2 + [ctypes.c_int] * 3 + [ctypes.c_void_p] * 2
    dev = torch.device("cuda")
    M, K = 47232, 2048
    nbuf = 4
    As = [torch.randn(M, K, device=dev).half() for _ in range(nbuf)]
    B = torch.randn(512, K, device=dev).half()
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ntiles = (M // 192) * 2
    staged = ntiles * (K * 2 // 128) * (192 + 256) * 128  # bytes into LDS per launch
    for grid in (256, 512):
        for mode, depth in ((0, 2), (30, 2), (31, 2), (32, 2), (33, 2), (34, 2), (35, 2)):
            rc = lib.stage_lab(mode, depth, As[0].data_ptr(), B.data_ptr(), M, K, grid, sink.data_ptr(), st)
            if rc:
                print(f"mode {mode} depth {depth}: rc {rc}")
                continue
            best = 1e9
            for _ in range(3):
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for i in range(10):
                    lib.stage_lab(mode, depth, As[i % nbuf].data_ptr(), B.data_ptr(), M, K, grid, sink.data_ptr(), st)
                e.record()
                torch.cuda.synchronize()
                best = min(best, s.elapsed_time(e) / 10)
            print(f"grid {grid} {NAMES[mode]:32s} depth {depth}: {best * 1e3:7.1f} us  "
                  f"{staged / best / 1e9:6.2f} TB/s = {staged / best / 1e6 / 256:5.1f} GB/s per CU", flush=True)


if __name__ == "__main__":
    main()
