"""Per-step view of a rocprofv3 kernel trace (CSV): step boundaries at the last SGD kernel of
each step, then per stream the busy time, the idle gaps between kernels and the kernel classes
that take the time.

    python tools/trace_steps.py gpurun_out/prof_b1/p_kernel_trace.csv [--skip 3] [--steps 10]
"""
import argparse
import collections
import csv
import re


def short(name):
    m = re.search(r"clipk(?:::|\d+)(\w+?)(?:I|\(|E|$)", name)
    base = m.group(1) if m else name[:40]
    if "gemm_nt_kernel" in name:
        t = re.search(r"Li(\d+)ELi(\d+)ELi(\d+)E", name)
        base += f"<epi{t.group(1)},{t.group(2)}x{t.group(3)}>" if t else ""
    return base


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sgd = [i for i, r in enumerate(rows) if "sgd" in r["Kernel_Name"].lower()]
    # the last SGD launch of a step: followed by a gap of more than 0.2 ms to the next SGD launch
    ends = [i for k, i in enumerate(sgd)
            if k + 1 == len(sgd) or int(rows[sgd[k + 1]]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"]) > 200_000]
    ends = ends[a.skip:a.skip + a.steps + 1]
    n = len(ends) - 1
    t0, t1 = int(rows[ends[0]]["End_Timestamp"]), int(rows[ends[-1]]["End_Timestamp"])
    seg = [r for r in rows if t0 < int(r["Start_Timestamp"]) <= t1]
    print(f"{n} steps, {(t1 - t0) / n / 1e6:.3f} ms/step, {len(seg) / n:.0f} kernels/step")
    by = collections.defaultdict(list)
    for r in seg:
        by[r["Stream_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    for sid, ks in sorted(by.items()):
        ks.sort()
        busy, gap, ce = 0, 0, None
        cls = collections.defaultdict(lambda: [0, 0])
        for s, e, nm in ks:
            if ce is not None and s > ce:
                gap += s - ce
            busy += e - s if ce is None or s >= ce else max(0, e - ce)
            ce = e if ce is None else max(ce, e)
            c = cls[short(nm)]
            c[0] += 1
            c[1] += e - s
        print(f"stream {sid}: {len(ks) / n:.0f} kernels/step, busy {busy / n / 1e6:.3f} ms/step, "
              f"gaps {gap / n / 1e6:.3f} ms/step")
        for k, (c, t) in sorted(cls.items(), key=lambda kv: -kv[1][1])[:14]:
            print(f"   {k:45s} {c / n:6.1f}/step {t / n / 1e3:8.1f} us/step {t / c / 1e3:7.1f} us avg")


if __name__ == "__main__":
    main()
