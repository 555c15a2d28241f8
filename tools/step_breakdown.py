"""Per-training-step kernel breakdown from a rocprofv3 kernel-trace CSV of bench.py:
kernels between the first and the last sgd_kernel launch of the timed steps, grouped by
name. Usage: step_breakdown.py <p_kernel_trace.csv> <n_steps_timed>"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = int(sys.argv[2])
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the optimizer step closes each train step: sgd_multi_kernel (one per param group, round 4)
    # or the per-tensor sgd_kernel launches of earlier builds
    sgd = [i for i, r in enumerate(rows) if "sgd_kernel" in r["Kernel_Name"] or "sgd_multi_kernel" in r["Kernel_Name"]]
    per = len(sgd) // (steps + 3) if len(sgd) % (steps + 3) == 0 else None
    # the timed region: after the warmup steps' last sgd launch, up to the last sgd launch
    k = per or 1
    beg = sgd[-steps * k - 1] + 1
    end = sgd[-1] + 1
    agg = defaultdict(lambda: [0, 0.0])
    for r in rows[beg:end]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        a = agg[r["Kernel_Name"][:110]]
        a[0] += 1
        a[1] += d
    tot = sum(v[1] for v in agg.values())
    wall = (int(rows[end - 1]["End_Timestamp"]) - int(rows[beg]["Start_Timestamp"])) / 1e3
    print(f"per step: kernel busy {tot / steps / 1e3:.3f} ms, wall {wall / steps / 1e3:.3f} ms")
    for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"{d / steps:9.1f} us/step {100 * d / tot:5.1f}% {c // steps:4d}x {d / c:8.1f} us  {n}")


if __name__ == "__main__":
    main()
