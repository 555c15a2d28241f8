# batch-1 fp32s step (the reference's CoCoOp batch) under rocprofv3: where its 4.6 ms go
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06u
BATCH=1 PREC=fp32s MODE=vit timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06u/prof -o p -- python3 -u tools/lab/vit_contention.py 30 > gpurun_out/r06u/prof.log 2>&1
