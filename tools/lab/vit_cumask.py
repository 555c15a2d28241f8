"""The side-stream ViT prefetch on a CU-masked HIP stream (hipExtStreamCreateWithCUMask): does
keeping the frozen image encoder on a subset of the CUs cut what it costs the text chain?
Per (batch, classes, every-k-th CU): bench.time_train with the trainer's side stream replaced.
    python tools/lab/vit_cumask.py [1/1000,1/125,8/1000] [0,2,4,8]   (0 = unmasked stream)"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def masked_stream(torch, every):
    hip = ctypes.CDLL("libamdhip64.so")
    n = torch.cuda.get_device_properties(0).multi_processor_count
    words = (n + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for i in range(n):
        if i % every == 0:
            mask[i // 32] |= 1 << (i % 32)
    st = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return torch.cuda.ExternalStream(st.value, device=torch.device("cuda", 0)), sum(1 for i in range(n) if i % every == 0)


def main():
    import torch
    import bench
    cases = sys.argv[1] if len(sys.argv) > 1 else "1/1000,1/125,8/1000"
    everys = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,2,4,8").split(",")]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    streams = {e: masked_stream(torch, e) for e in everys if e}
    for tok in cases.split(","):
        b, c = (int(x) for x in tok.split("/"))
        tr, dm = bench.build_trainer(argparse.Namespace(arch="ViT-B/16", classes=c), "fp16", b, dev, 0)
        n = 50 if b == 1 else 20
        line = f"B {b} C {c:5d}:"
        for rnd in range(2):
            for e in everys:
                if e:
                    tr.model._side_stream = streams[e][0]
                else:
                    tr.model._side_stream = None
                t = bench.time_train(tr, dm, n, 5)[0]
                line += f" | {('all' if not e else str(streams[e][1]) + ' CUs'):>7s} {1000 * t / n:.3f}"
        print(line + " ms/step", flush=True)
        del tr, dm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
