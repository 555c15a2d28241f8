# kernel traces of the batch-1 125-class step alone and right after a ViT-L/14 B=32 trainer
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05o; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/alone -o t -- python3 $GRAFT_REPO_ROOT/tools/lab/proxy_order.py 125 > $O/alone.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/after -o t -- python3 $GRAFT_REPO_ROOT/tools/lab/proxy_order.py 1000/32/bf16/ViT-L/14,125 > $O/after.log 2>&1 || exit $?
echo ok
