# round-4 GPU pass x: main-stream priority vs the side-stream ViT (tools/prio_time.py), B = 8 and 1
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/prio_time.py --batch 8 > gpurun_out/r04x_prio.txt 2>&1 && \
timeout -k 10 300 python -u tools/prio_time.py --batch 1 --steps 100 >> gpurun_out/r04x_prio.txt 2>&1
rc=$?
echo exit $rc
exit $rc
