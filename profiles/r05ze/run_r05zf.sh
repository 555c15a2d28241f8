# PMC view of the headline step's kernels (bench workload): MFMA / TA / TD / LDS busy, L1 pending stalls
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05zf; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum --output-format csv -d $O/a -o p -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof --no-extra --eval-images 0 > $O/a.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $O/b -o p -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof --no-extra --eval-images 0 > $O/b.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $O/t -o p -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof --no-extra --eval-images 0 > $O/t.log 2>&1 || exit $?
echo ok
