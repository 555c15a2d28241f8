# where fp32s eval time goes: 2,000 images (test batch 100) under rocprofv3 --kernel-trace --stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06r
PREC=fp32s timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06r/prof -o p -- python3 -u tools/lab/eval_parts.py 2000 > gpurun_out/r06r/prof.log 2>&1
