"""hipBLASLt on the step's text GEMM shapes (M = 47,160 packed rows, fp16 in / fp16 out, NT):
run under `rocprofv3 --kernel-trace --stats` to read which kernel (macro tile, MFMA shape,
workgroup) the library picks per shape, next to its rate from HIP events.
    python tools/lab/blaslt_shapes.py"""
import torch


def main():
    dev = torch.device("cuda")
    M = 47160
    g = torch.Generator(device=dev).manual_seed(0)
    for n, k in ((512, 2048), (512, 1536), (512, 512), (2048, 512), (1536, 512)):
        nbuf = max(2, -(-600_000_000 // (M * k * 2)))
        As = [(torch.randn(M, k, device=dev, generator=g) * 0.5).half() for _ in range(nbuf)]
        B = (torch.randn(n, k, device=dev, generator=g) * 0.5).half()
        C = torch.empty(M, n, device=dev, dtype=torch.float16)
        for i in range(3):
            torch.matmul(As[i % nbuf], B.t(), out=C)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for i in range(12):
            torch.matmul(As[i % nbuf], B.t(), out=C)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 12
        print(f"N{n} K{k}: hipBLASLt {ms * 1e3:7.1f} us {2.0 * M * n * k / ms / 1e9:7.1f} TF/s", flush=True)
        del As, B, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
