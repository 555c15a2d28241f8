# round 5: MFMA yardstick, eval chunk sweep, GEMM tile sweep on the N = 512 shapes
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 120 python -u tools/lab/mfma_peak.py > $O/mfma_peak.txt 2>&1 && \
timeout -k 10 300 python -u tools/eval_chunk_sweep.py fp16 > $O/eval_chunk.txt 2>&1 && \
for c in 6 1 2 0; do
  CLIPK_GEMM_CFG=$c timeout -k 10 200 python -u tools/gemm_yardstick.py --no-ref --only out_dx >> $O/cfg_sweep.txt 2>&1 || exit $?
  CLIPK_GEMM_CFG=$c timeout -k 10 200 python -u tools/gemm_yardstick.py 8000 --no-ref --only out_dx >> $O/cfg_sweep.txt 2>&1 || exit $?
  CLIPK_GEMM_CFG=$c timeout -k 10 200 python -u tools/gemm_yardstick.py 8000 --no-ref --only fc_dx >> $O/cfg_sweep.txt 2>&1 || exit $?
  echo "cfg $c done" >> $O/cfg_sweep.txt
done
echo exit $?
