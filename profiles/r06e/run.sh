# round 6: ATen launches folded into clipk kernels (Meta-Net norm, CE reduce, ctx/bias sums, status take,
# unit-grad backward), ViT prefetch queued after the forward; tests + bench + step parts + ATen census
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_split_w16_gpu.py tests/test_trainer_gpu.py tests/test_vision_schedule_gpu.py tests/test_dist_nccl_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_kern.txt 2>&1 || { echo "kernel/trainer tests failed"; tail -30 $O/t_kern.txt; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q -k "cocoop or headline or prefix_input" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_parity.txt 2>&1 || { echo "parity failed"; tail -30 $O/t_parity.txt; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 50000 > $O/b_1.json 2> $O/b_1.err || exit 1
PREC=fp32s timeout -k 10 500 python -u tools/lab/step_parts.py 8/1000,1/1000 > $O/step_parts.txt 2> $O/step_parts.err || exit 1
timeout -k 10 300 python -u tools/aten_on_step.py > $O/aten_on_step.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 5000 > $O/b_2.json 2> $O/b_2.err || exit 1
echo done
