"""MFMA throughput the chip sustains (tools/lab/mfma_peak.hip): 16x16x32 f16 MFMAs back to back
on register operands, every CU busy, one and two waves per SIMD, random and zero operands; TF/s
from HIP events and the in-kernel clock (s_memtime / s_memrealtime x 100 MHz).
    python tools/lab/mfma_peak.py"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libmfmapeak.so"))
    lib.mfma_peak.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                              ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    blocks, iters = 256, 20000
    clk = torch.zeros(2, dtype=torch.int64, device=dev)
    for data in ("random", "zeros"):
        src = (torch.randn(256, 8, device=dev) if data == "random" else torch.zeros(256, 8, device=dev)).half()
        for wps in (1, 2):
            out = torch.empty(blocks * 256 * wps, device=dev)
            for _ in range(3):  # warm the clock up (DVFS), then time
                lib.mfma_peak(wps, src.data_ptr(), out.data_ptr(), iters, blocks, clk.data_ptr(), st)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            n = 5
            for _ in range(n):
                lib.mfma_peak(wps, src.data_ptr(), out.data_ptr(), iters, blocks, clk.data_ptr(), st)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / n
            flops = 2.0 * 16 * 16 * 32 * 8 * iters * 4 * wps * blocks  # per wave: 8 MFMAs per iteration
            c = clk.cpu().tolist()
            ghz = c[0] / (c[1] / 100e6) / 1e9 if c[1] else 0.0
            print(f"{data:6s} waves/SIMD {wps}: {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TF/s  "
                  f"({flops / ms / 1e9 / 2500:.3f} of 2.5 PF)  in-kernel clock {ghz:.2f} GHz", flush=True)


if __name__ == "__main__":
    main()
