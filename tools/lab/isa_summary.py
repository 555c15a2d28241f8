"""Compact instruction timeline of one kernel in a .s file: runs of instruction classes.
    python isa_summary.py file.s kernel_symbol_substring"""
import re
import sys

src, key = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_") and key in l and l.split(";")[0].strip().endswith(":"))
body = []
for l in lines[start + 1:]:
    if l.strip().startswith("s_endpgm"):
        break
    body.append(l)


def cls(l):
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        return None
    if t.endswith(":"):
        return "LABEL " + t
    op = t.split()[0]
    for p in ("v_mfma", "ds_read", "ds_write", "global_load_lds", "global_load", "global_store", "buffer_store",
              "buffer_load", "scratch", "s_barrier", "s_waitcnt", "s_cbranch", "v_accvgpr_write", "v_accvgpr_read",
              "s_setprio", "s_nop"):
        if op.startswith(p):
            return op if p in ("s_waitcnt",) else p
    return "valu" if op.startswith("v_") else "salu"


runs = []
for l in body:
    c = cls(l)
    if c is None:
        continue
    if c == "s_waitcnt":
        c = l.strip()
    if runs and runs[-1][0] == c and not c.startswith("LABEL"):
        runs[-1][1] += 1
    else:
        runs.append([c, 1])
print(" | ".join(f"{c}x{n}" if n > 1 else c for c, n in runs))
