# round-4 GPU pass: what the side-stream ViT costs the train step (tools/vit_cost.py), B = 8 and 1
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/vit_cost.py --batch 8 > gpurun_out/r04z4_vitcost.txt 2>&1 && \
timeout -k 10 300 python -u tools/vit_cost.py --batch 1 --steps 100 >> gpurun_out/r04z4_vitcost.txt 2>&1
rc=$?
echo exit $rc
exit $rc
