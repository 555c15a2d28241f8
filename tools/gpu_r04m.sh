# round-4 GPU pass m: LN statistics merge with 4 rows per lane group (lnfold tests), the eval
# site table and the headline bench against the previous merge (build_ab/merge0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lnfold_gpu.py \
  > gpurun_out/r04m_lnfold.txt 2>&1 && \
timeout -k 10 300 python -u tools/eval_sites.py > gpurun_out/r04m_eval1.txt 2>&1 && \
CLIPK_LIB=build_ab/merge0/libclipk.so timeout -k 10 300 python -u tools/eval_sites.py > gpurun_out/r04m_eval0.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline --no-configs --eval-images 5000 --steps 20 > gpurun_out/r04m_b1.json 2>/dev/null && \
CLIPK_LIB=build_ab/merge0/libclipk.so timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline --no-configs --eval-images 5000 --steps 20 > gpurun_out/r04m_b0.json 2>/dev/null
rc=$?
echo exit $rc
exit $rc
