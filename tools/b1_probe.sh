#!/bin/bash
# batch-1 train step (the reference's CoCoOp batch): kernel-class table under tile-config knobs
mkdir -p gpurun_out
IFS=";" read -ra VS <<< "${VARIANTS:-base}"
for v in "${VS[@]}"; do
  [ "$v" = base ] && v=""
  env $v timeout -k 10 200 python -u bench.py --batch 1 --steps 30 --warmup 5 --no-extra --no-cpu-baseline \
    --eval-images 0 > gpurun_out/b1_probe.json 2>> gpurun_out/b1_err.log || exit 1
  tail -1 gpurun_out/b1_probe.json | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']
print('[$v]', 'ms', d['ms_per_step'], ' '.join(f'{n}={v[\"ms_per_step\"]:.3f}' for n,v in k.items()))
" | tee -a gpurun_out/b1.log
done
