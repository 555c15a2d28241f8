# round-4 GPU pass y: Meta-Net forward over (image, 64-output) blocks + one multi-tensor SGD
# launch per param group: kernel / trainer / parity tests, then the batch-1 kernel trace
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "meta" \
  > gpurun_out/r04y3_tests.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_trainer_gpu.py tests/test_parity_gpu.py \
  >> gpurun_out/r04y3_tests.txt 2>&1 && \
timeout -k 10 120 python -u tools/b1_time.py > gpurun_out/r04y3_b1.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r04y3_tr -o p -- python3 $R/tools/cpu_issue_probe.py --batches 1 --steps 20 > $R/gpurun_out/r04y3_tr.log 2>&1 && \
cd $R && python3 tools/trace_steps.py gpurun_out/r04y3_tr/p_kernel_trace.csv --skip 3 --steps 10 > gpurun_out/r04y3_b1_trace.txt 2>&1
rc=$?
echo exit $rc
exit $rc
