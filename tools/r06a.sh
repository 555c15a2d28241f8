set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_split_w16_gpu.py tests/test_lnfold_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_split.txt 2>&1 || { echo "split tests rc $?"; exit 1; }
timeout -k 10 300 python -u bench.py --prec fp32s --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 5000 > $O/b_fp32s.json 2> $O/b_fp32s.err
timeout -k 10 300 env FSP_SPLIT_W16=0 python -u bench.py --prec fp32s --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 5000 > $O/b_fp32s_mode1.json 2> $O/b_fp32s_mode1.err
timeout -k 10 300 python -u bench.py --prec fp32s --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 5000 > $O/b_fp32s_2.json 2> $O/b_fp32s_2.err
echo done
