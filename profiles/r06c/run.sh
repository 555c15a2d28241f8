# round 6: pre-split dq|dk|dv (DPP-paired 16-B stores), split asm with its own wait states
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_split_w16_gpu.py tests/test_kernels_gpu.py -k "split or prefix or gemm" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_split.txt 2>&1 || { echo "split tests failed"; tail -30 $O/t_split.txt; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q -k "fp32s or w16 or prefix_input" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_parity.txt 2>&1 || { echo "parity failed"; tail -30 $O/t_parity.txt; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 5000 > $O/b_on_$r.json 2> $O/b_on_$r.err || exit 1
timeout -k 10 300 env CLIPK_PRESPLIT_QKV=0 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 5000 > $O/b_off_$r.json 2> $O/b_off_$r.err || exit 1
done
echo done
