# round-4 GPU pass k: c_fc saves quickgelu'(h) (CLIPK_QGELU_DERIV) -- kernel tests, the encoder /
# trainer parity suites that run the text and prompted-ViT backward, then the headline step's
# site table with the derivative form on / off (CLIPK_QGELU_DERIV=0), interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py -k "qgelu_deriv or splitk or epilogues" tests/test_lnfold_gpu.py \
  > gpurun_out/r04k_tests.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_parity_gpu.py tests/test_deep_gpu.py tests/test_trainer_gpu.py > gpurun_out/r04k_parity.txt 2>&1 && \
timeout -k 10 300 python -u tools/site_table.py > gpurun_out/r04k_d1.txt 2>&1 && \
CLIPK_QGELU_DERIV=0 timeout -k 10 300 python -u tools/site_table.py > gpurun_out/r04k_d0.txt 2>&1 && \
timeout -k 10 300 python -u tools/site_table.py >> gpurun_out/r04k_d1.txt 2>&1 && \
CLIPK_QGELU_DERIV=0 timeout -k 10 300 python -u tools/site_table.py >> gpurun_out/r04k_d0.txt 2>&1 \
  && timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline --no-configs --eval-images 0 --steps 20 > gpurun_out/r04k_b1.json 2>/dev/null && \
CLIPK_QGELU_DERIV=0 timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline --no-configs --eval-images 0 --steps 20 > gpurun_out/r04k_b0.json 2>/dev/null
rc=$?
echo exit $rc
exit $rc
