# batch-1 graph probe: eager vs HIP-graph replay of the CoCoOp train step (fp16 and fp32s)
set -o pipefail
mkdir -p gpurun_out/r06l
timeout -k 10 300 python -u tools/graph_probe.py --batch 1 --prec fp16 --steps 50 2>&1 | tee gpurun_out/r06l/graph_b1_fp16.txt &&
timeout -k 10 300 python -u tools/graph_probe.py --batch 1 --prec fp32s --steps 50 2>&1 | tee gpurun_out/r06l/graph_b1_fp32s.txt
