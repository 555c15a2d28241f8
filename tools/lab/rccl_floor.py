"""Per-step collectives of the multi-GPU paths, timed in a 1-rank RCCL group on one GPU: the
gradient all-reduce (dist.allreduce_grads: ctx + Meta-Net, 35,360 fp32 = 138 KB, one flat
bucket) and the class-sharded CoCoOp logits all-gather ([B, C/N] fp32). One rank moves no data
over xGMI, so this is each call's fixed cost (launch, RCCL's own kernel, host), the floor under
the N-rank figure. HIP events around 200 back-to-back calls.
    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 \
        tools/lab/rccl_floor.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fsp_amd import dist  # noqa: E402


def timeit(fn, n=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    local = dist.init_from_env("nccl")
    dev = torch.device("cuda", local)
    shapes = {"ctx": (4, 512), "w1": (32, 512), "b1": (32,), "w2": (512, 32), "b2": (512,)}
    ps = [torch.nn.Parameter(torch.randn(*s, device=dev)) for s in shapes.values()]
    for p in ps:
        p.grad = torch.randn_like(p)

    def ar():
        dist.allreduce_grads(ps)

    print(f"world {dist.world_size()}: allreduce_grads (138 KB, flat bucket) {timeit(ar):.1f} us/call", flush=True)
    flat = torch.randn(sum(p.numel() for p in ps), device=dev)
    print(f"world {dist.world_size()}: bare all_reduce of 138 KB {timeit(lambda: torch.distributed.all_reduce(flat)):.1f} us/call",
          flush=True)
    for b, c in ((1, 125), (1, 1000), (8, 125)):
        x = torch.randn(b, c, device=dev)
        counts = [c] * dist.world_size()
        t = timeit(lambda: dist.GatherClassColumns.apply(x, counts))
        print(f"world {dist.world_size()}: logits all-gather [B {b}, C_r {c}] {t:.1f} us/call", flush=True)
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
