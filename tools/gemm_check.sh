set -e
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k gemm > gpurun_out/t_gemm.log 2>&1
KB_M=47160 KB_CFGS=1,6,2 KB_ONLY=gemm timeout -k 10 120 python -u tools/kbench.py > gpurun_out/kb9.log 2>&1
bash tools/pmc_bench.sh gpurun_out/pmc_bench > gpurun_out/pmc.log 2>&1
