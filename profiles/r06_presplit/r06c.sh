set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_split_w16_gpu.py tests/test_lnfold_gpu.py -x -q -rs --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_split.txt 2>&1 || { echo "split tests failed"; tail -30 $O/t_split.txt; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -x -q -k "fp32s or w16" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_parity_fp32s.txt 2>&1 || { echo "parity failed"; tail -30 $O/t_parity_fp32s.txt; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --prec fp32s --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 5000 > $O/b_fp32s_$r.json 2> $O/b_fp32s_$r.err
timeout -k 10 300 env CLIPK_PRESPLIT=0 python -u bench.py --prec fp32s --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 5000 > $O/b_fp32s_nops_$r.json 2> $O/b_fp32s_nops_$r.err
done

timeout -k 10 300 python -u tools/aten_on_step.py > gpurun_out/r06c/aten_on_step.txt 2>&1
echo done
