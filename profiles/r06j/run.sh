# round 6: PREC fp32s ViT on the layer loop (LayerNorm fold with gamma on A, pre-split hand-offs, last layer
# on the CLS rows), second try (the patch embedding's GEMM inside the split scope): a focused parity run first,
# then the ViT-touching suites and an A/B bench against CLIPK_VIT_LOOP32=0
set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -k "cocoop_full and fp32s" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t_first.txt 2>&1 || { echo "focused parity failed"; tail -20 $O/t_first.txt; exit 1; }
timeout -k 10 700 python -u -m pytest tests/test_parity_gpu.py tests/test_deep_gpu.py tests/test_vision_schedule_gpu.py tests/test_split_w16_gpu.py tests/test_lnfold_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_vit.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 5000 > $O/b_on_$r.json 2> $O/b_on_$r.err || exit 1
timeout -k 10 240 env CLIPK_VIT_LOOP32=0 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 5000 > $O/b_off_$r.json 2> $O/b_off_$r.err || exit 1
done
echo done
