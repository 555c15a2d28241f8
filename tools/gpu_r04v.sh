# round-4 GPU pass v: fp32 LayerNorm forward rows per wave (CLIPK_LN_RPW32 = 1 / 2 / 4): LN
# tests under each, then the fp32s site table per setting
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 4; do
  CLIPK_LN_RPW32=$r timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k layernorm \
    >> gpurun_out/r04v_tests.txt 2>&1 || exit 1
done
for r in 2 4 1 2 4; do
  echo "== CLIPK_LN_RPW32=$r" >> gpurun_out/r04v_sites.txt
  CLIPK_LN_RPW32=$r timeout -k 10 300 python -u tools/site_table.py --prec fp32s 2>&1 | grep -E "sum of|ln_fwd|ln_bwd" >> gpurun_out/r04v_sites.txt || exit 1
done
echo exit 0
