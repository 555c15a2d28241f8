# TD / TA / MFMA busy of the fc_dx product: the production kernel (LDS-DMA staging) vs hipBLASLt
# (register-staged global reads) on the same shape
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05zg; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ours blaslt; do
  B=""; [ $v = blaslt ] && B=1
  BLASLT=$B timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum --output-format csv -d $O/$v -o p -- python3 $R/tools/lab/gemm_only.py > $O/$v.log 2>&1 || exit $?
  BLASLT=$B timeout -s KILL 90 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $O/${v}_b -o p -- python3 $R/tools/lab/gemm_only.py > $O/${v}_b.log 2>&1 || exit $?
done
echo ok
