"""Register / spill / LDS usage of the kernels in a built object (code-object metadata notes).

    python tools/kernel_regs.py <build/xxx.o> [name-substring ...]

Extracts the gfx950 code object from the object's .hip_fatbin section (llvm-objcopy +
clang-offload-bundler) and prints vgpr / agpr / spill counts and static LDS per kernel."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernel_regs(obj):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "g.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "x.o")],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    rows = []
    for e in notes.split(".name:")[1:]:
        name = e.split("\n")[0].strip()

        def g(k):
            m = re.search(r"\." + k + r":\s+(\d+)", e)
            return int(m.group(1)) if m else None
        rows.append({"name": name, "vgpr": g("vgpr_count"), "agpr": g("agpr_count"),
                     "vgpr_spill": g("vgpr_spill_count"), "sgpr_spill": g("sgpr_spill_count"),
                     "lds": g("group_segment_fixed_size")})
    return rows


if __name__ == "__main__":
    pats = sys.argv[2:]
    for r in kernel_regs(sys.argv[1]):
        if not pats or all(p in r["name"] for p in pats):
            print(f"vgpr {r['vgpr']:4} agpr {r['agpr']:4} vspill {r['vgpr_spill']:3} sspill {r['sgpr_spill']:3} "
                  f"lds {r['lds']:6}  {r['name'][:150]}")
