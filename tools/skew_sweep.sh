set -e
for sk in 0 4 8 16; do
  echo "=== skew $sk" >> gpurun_out/kb3.log
  CLIPK_GEMM_SKEW=$sk KB_M=47160 KB_CFGS=4,5 KB_ONLY=gemm timeout -k 10 120 python -u tools/kbench.py >> gpurun_out/kb3.log 2>&1
done
