# PMC view of the N = 512 K = 2048 input-grad GEMM alone: MFMA / TA / TD / LDS busy and TCP stalls
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05ze; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum --output-format csv -d $O/a -o p -- python3 $R/tools/lab/gemm_only.py > $O/a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $O/b -o p -- python3 $R/tools/lab/gemm_only.py > $O/b.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/t -o p -- python3 $R/tools/lab/gemm_only.py > $O/t.log 2>&1 || exit $?
echo ok
