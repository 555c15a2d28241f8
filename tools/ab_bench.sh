#!/bin/bash
# A/B of library variants on the headline bench (GPU box): tools/ab_bench.sh tag1 tag2 ...
# ("base" = the in-tree libclipk.so; "env:NAME=VAL[,NAME=VAL]" = the in-tree library with those
# runtime knobs; others build_ab/<tag>/libclipk.so). Two interleaved rounds; one summary line
# per run in gpurun_out/ab.log.
R=$(pwd)
mkdir -p gpurun_out
for round in 1 2; do
  for t in "$@"; do
    L=""; ENVS=""
    case $t in
      base) ;;
      env:*) ENVS=${t#env:}; ENVS=${ENVS//,/ };;
      *) L=$R/build_ab/$t/libclipk.so;;
    esac
    f=gpurun_out/ab_$(echo "$t" | tr -c 'A-Za-z0-9_\n' '_')_${round}.json
    env $ENVS CLIPK_LIB=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline \
      --eval-images 2000 > $f 2> gpurun_out/ab_err.log || exit 1
    tail -1 $f | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']
print('$t', $round, 'ms', d['ms_per_step'], 'eval', round(d['eval_images_per_sec']), ' '.join(f'{n}={v[1]:.3f}' for n,v in k.items()))
" | tee -a gpurun_out/ab.log
  done
done
