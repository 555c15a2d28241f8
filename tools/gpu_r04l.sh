# round-4 GPU pass l: the LN-fold kernel tests (incl. the QuickGELU-derivative fold form), and
# where the eval forward's time goes (site table + rocprofv3 kernel stats of eval alone)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lnfold_gpu.py \
  > gpurun_out/r04l_lnfold.txt 2>&1 && \
timeout -k 10 300 python -u tools/eval_sites.py > gpurun_out/r04l_eval_sites.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04l_evprof -o p -- \
  python3 $R/tools/eval_sites.py --batches 3 > $R/gpurun_out/r04l_evprof.log 2>&1
rc=$?
echo exit $rc
exit $rc
