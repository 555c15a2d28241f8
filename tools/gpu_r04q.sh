# round-4 GPU pass q: where the fp32 prefix-attention kernels spend their cycles -- isolated
# timing, then SQ counters (one rocprofv3 --pmc pass each) of the same run
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r04q
SWEEP_DTYPE=fp32 timeout -k 10 120 python -u tools/attn_sweep.py --one > gpurun_out/r04q/time.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
SWEEP_DTYPE=fp32 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/r04q/p1 -o p -- python3 $R/tools/attn_sweep.py --one > $R/gpurun_out/r04q/p1.log 2>&1 && \
SWEEP_DTYPE=fp32 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/r04q/p2 -o p -- python3 $R/tools/attn_sweep.py --one > $R/gpurun_out/r04q/p2.log 2>&1
rc=$?
echo exit $rc
exit $rc
