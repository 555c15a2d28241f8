"""ViT attention forward A/B (HIP events, isolated launches): the step's shapes -- B/16 at 8
images (L 197, 12 heads), L/14@336 at 8 images (L 577, 16 heads), B/16 eval at 100 images --
for the kernel the library picks (attn_fwd_mfma_t). Prints us per launch and the fraction of the HBM roofline for the
algorithmic bytes (read q|k|v, write o, 16-bit)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd import ops  # noqa: E402
from tools.kbench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    tag = os.environ.get("AB_TAG", "fwd")
    for nseq, L, H in ((8, 197, 12), (8, 577, 16), (100, 197, 12), (8, 50, 12)):
        g = torch.Generator(device="cpu").manual_seed(L)
        qkv = torch.randn(nseq * L, 3 * H * 64, generator=g).to(dev, torch.float16)
        t = timeit(lambda: ops.attention(qkv, nseq, L, H, 0), iters=20)
        byt = nseq * L * 4 * H * 64 * 2
        fl = 4.0 * nseq * H * L * L * 64
        print(f"{tag} nseq {nseq:4d} L {L:4d} H {H:3d}: {t * 1e3:7.1f} us  {byt / t / 1e6:7.1f} GB/s  "
              f"{fl / t / 1e9:6.1f} TF/s")


if __name__ == "__main__":
    main()
