"""Per-kernel HBM traffic from the two PMC passes of tools/pmc_bench.sh.
FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB; on gfx950 FETCH_SIZE counts
128-B requests at 64 B (MI355X_MICROARCH.md, HBM), so it is doubled here."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    agg = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    d = sys.argv[1]
    fe, wr = load(os.path.join(d, "fetch"), "FETCH_SIZE"), load(os.path.join(d, "write"), "WRITE_SIZE")
    rows = []
    for k in set(fe) | set(wr):
        f = sum(fe.get(k, [0])) / max(len(fe.get(k, [])), 1)
        w = sum(wr.get(k, [0])) / max(len(wr.get(k, [])), 1)
        rows.append((2 * f * 1024 + w * 1024, 2 * f * 1024, w * 1024, len(fe.get(k, [])), k))
    rows.sort(reverse=True)
    out = {}
    print("hbm_bytes_per_launch, fetch_x2, write, launches, kernel")
    for t, f, w, n, k in rows[:25]:
        print(f"{t:.4e}, {f:.4e}, {w:.4e}, {n}, {k[:110]}")
        out[k] = {"hbm_bytes": t, "fetch_bytes_x2": f, "write_bytes": w, "launches": n}
    json.dump(out, open(os.path.join(d, "traffic.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
