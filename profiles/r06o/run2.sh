# kernel stats of the fp32s step with the ViT in line (serial) and with cached features (novit):
# the difference is the ViT forward's standalone kernels at 8 images
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06o
for m in serial novit; do
  PREC=fp32s MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06o/prof_$m -o p -- python3 -u tools/lab/vit_contention.py 10 > gpurun_out/r06o/prof_$m.log 2>&1 || exit 1
done
