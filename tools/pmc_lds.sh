#!/bin/bash
# LDS-side PMC pass over one GEMM shape (tools/one_gemm.py): bank conflicts, LDS-array busy
# cycles and unaligned replays next to MFMA-busy and wave cycles (one counter pass per shape).
set -e
R=$(pwd)
OUT=$R/gpurun_out/pmc_lds
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for shape in plain fcbwd; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/$shape -o p -- python3 $R/tools/one_gemm.py $shape 5 > $OUT/$shape.log 2>&1
done
python3 - <<'PY'
import csv, glob, collections
for shape in ("plain", "fcbwd"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"/root/repo/gpurun_out/pmc_lds/{shape}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemm_nt" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    print(shape, {k: f"{v:.4g}" for k, v in sorted(m.items())})
    busy = m.get("SQ_BUSY_CYCLES", 1)
    print("  per SQ-busy cycle: mfma-busy %.3f  lds-array %.3f  bank-conflict %.3f  unaligned %.3f" % (
        m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / busy, m.get("SQ_LDS_IDX_ACTIVE", 0) / busy,
        m.get("SQ_LDS_BANK_CONFLICT", 0) / busy, m.get("SQ_LDS_UNALIGNED_STALL", 0) / busy))
PY
