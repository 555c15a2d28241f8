# round-4: fp32 prefix attention waves per block (CLIPK_F32ATTN_WPB 2 = default, 4, 8) on the
# interleaved column map, isolated fwd / bwd at the bench shape
set -o pipefail
mkdir -p gpurun_out
for v in 2 4 8 2 4 8; do
  echo "wpb$v $(CLIPK_F32ATTN_WPB=$v SWEEP_DTYPE=fp32 timeout -k 10 120 python -u tools/attn_sweep.py --one 2>/dev/null | grep rows)" >> gpurun_out/r04zd_attn.txt || exit 1
done
echo exit 0
