set -e
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k gemm > gpurun_out/t_gemm.log 2>&1
for e in 0 1; do
echo "=== PIPE $e" >> gpurun_out/kb8.log
CLIPK_GEMM_PIPE=$e KB_M=47160 KB_CFGS=1 KB_ONLY=gemm timeout -k 10 120 python -u tools/kbench.py >> gpurun_out/kb8.log 2>&1
done
CLIPK_GEMM_PIPE=1 KB_CFGS=1 KB_ONLY=ksweep timeout -k 10 200 python -u tools/kbench.py >> gpurun_out/kb8.log 2>&1
