#!/bin/bash
# SQ stall split and L2 behaviour of the shared-prefix attention kernels at the bench shape
# (tools/kbench.py KB_ONLY=prefix), one counter group per rocprofv3 --pmc pass.
set -e
R=$(pwd)
OUT=$R/gpurun_out/pmc_attn
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export KB_ONLY=prefix
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o p -- python3 $R/tools/kbench.py > $OUT/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/tcc -o p -- python3 $R/tools/kbench.py > $OUT/tcc.log 2>&1 || true
python3 - <<'PY'
import csv, glob, collections
for grp in ("sq", "tcc"):
    for kern in ("attn_prefix_fwd", "attn_prefix_bwd"):
        agg = collections.defaultdict(list)
        for f in glob.glob(f"/root/repo/gpurun_out/pmc_attn/{grp}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if kern in r["Kernel_Name"]:
                    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        m = {k: sum(v) / len(v) for k, v in agg.items()}
        print(grp, kern, {k: f"{v:.4g}" for k, v in sorted(m.items())})
        if grp == "sq" and m:
            wc = m.get("SQ_WAVE_CYCLES", 1)
            print("   wait_any %.3f wait_inst %.3f active %.3f" % (m.get("SQ_WAIT_ANY", 0) / wc,
                  m.get("SQ_WAIT_INST_ANY", 0) / wc, m.get("SQ_ACTIVE_INST_ANY", 0) / wc))
PY
