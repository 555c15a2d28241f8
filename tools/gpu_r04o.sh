# round-4 GPU pass o: batch-1 step (tools/b1_time.py) after the r04z bench's 3.32 ms: current
# build, QuickGELU derivative off, the previous LN-statistics merge (build_ab/merge0), interleaved
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python -u tools/b1_time.py >> gpurun_out/r04o_b1.txt 2>&1 || exit 1
  CLIPK_QGELU_DERIV=0 timeout -k 10 120 python -u tools/b1_time.py >> gpurun_out/r04o_b1.txt 2>&1 || exit 1
  CLIPK_LIB=build_ab/merge0/libclipk.so timeout -k 10 120 python -u tools/b1_time.py >> gpurun_out/r04o_b1.txt 2>&1 || exit 1
done
echo exit 0
