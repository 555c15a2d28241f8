# round 6: tests of the folded launches + group-0 class rows (layer 0), bench, step parts, ATen census,
# main-stream priority lab, PMC counters of the fp32 prefix attention kernels
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_split_w16_gpu.py tests/test_trainer_gpu.py tests/test_vision_schedule_gpu.py tests/test_dist_nccl_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_kern.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q -k "cocoop or headline or prefix_input" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_parity.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 50000 > $O/b_1.json 2> $O/b_1.err || exit 1
PREC=fp32s timeout -k 10 500 python -u tools/lab/step_parts.py 8/1000,1/1000 > $O/step_parts.txt 2> $O/step_parts.err || exit 1
timeout -k 10 300 python -u tools/aten_on_step.py > $O/aten_on_step.txt 2>&1 || exit 1
PREC=fp32s timeout -k 10 400 python -u tools/lab/stream_priority.py 8/1000,1/1000 > $O/stream_priority.txt 2> $O/stream_priority.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum --kernel-include-regex "attn_prefix" --output-format csv -d $O/pmc_attn_a -o p -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof --no-extra --eval-images 0 > $O/pmc_attn_a.log 2>&1 || exit 1
echo done
