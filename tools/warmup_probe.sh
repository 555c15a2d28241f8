#!/bin/bash
# headline step time vs warm-up length (same box, same process order)
mkdir -p gpurun_out
for wk in "3 10" "20 30" "3 10" "50 50"; do
  set -- $wk
  timeout -k 10 300 python -u bench.py --warmup $1 --steps $2 --no-extra --no-cpu-baseline --eval-images 0 --no-prof \
    > gpurun_out/wp.json 2>>gpurun_out/wp_err.log || exit 1
  tail -1 gpurun_out/wp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('warmup $1 steps $2', d['ms_per_step'], d['value'])" | tee -a gpurun_out/warmup.log
done
