# round-4 GPU pass t: 16-bit prefix-attention forward units per wave (CLIPK_PREFIX_FWD_CHUNK)
# around the default 4: 7,552 waves at 4 = 3.7 rounds of 2,048 resident; 5 -> 2.97 rounds
set -o pipefail
mkdir -p gpurun_out
for c in 4 5 6 3 4 5; do
  CLIPK_PREFIX_FWD_CHUNK=$c timeout -k 10 120 python -u tools/attn_sweep.py --one > gpurun_out/r04t_c$c.tmp 2>&1 || exit 1
  echo "chunk $c $(grep rows gpurun_out/r04t_c$c.tmp)" >> gpurun_out/r04t_fwd_chunk.txt
done
echo exit 0
