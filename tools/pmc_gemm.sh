#!/bin/bash
# SQ stall breakdown of one GEMM shape (tools/one_gemm.py), one counter pass.
set -e
R=$(pwd)
OUT=$R/gpurun_out/pmc_gemm
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for shape in plain fcbwd; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/$shape -o p -- python3 $R/tools/one_gemm.py $shape 5 > $OUT/$shape.log 2>&1
done
python3 - <<'PY'
import csv, glob, collections
for shape in ("plain", "fcbwd"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"/root/repo/gpurun_out/pmc_gemm/{shape}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemm_nt" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    print(shape, {k: f"{v:.4g}" for k, v in sorted(m.items())})
    wc = m.get("SQ_WAVE_CYCLES", 1)
    print("  wait_any %.3f  wait_inst %.3f  active %.3f  (of wave cycles); lds-issue-wait %.3f" % (
        m.get("SQ_WAIT_ANY", 0) / wc, m.get("SQ_WAIT_INST_ANY", 0) / wc, m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        m.get("SQ_WAIT_INST_LDS", 0) / wc))
PY
