# the fp32 prefix attention forward held to 4 waves per SIMD (CLIPK_PREFIX_F32_DEEP 3: 128 VGPRs,
# 52 B of scratch) against 3 (0): the prefix-attention tests, the fp32s step interleaved, rocprof
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06s
F='^>>\|Loading\|Use \|amdgpu.ids'
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "attention_prefix_kernel_variants" > gpurun_out/r06s/tests2.txt 2>&1 || { tail -30 gpurun_out/r06s/tests2.txt; exit 1; }
tail -1 gpurun_out/r06s/tests2.txt
for i in 1 2 3; do
  for d in 0 3; do
    echo "=== deep $d" >> gpurun_out/r06s/ab2.txt
    CLIPK_PREFIX_F32_DEEP=$d PREC=fp32s MODE=vit timeout -k 10 240 python -u tools/lab/vit_contention.py 30 2>&1 | grep -v "$F" >> gpurun_out/r06s/ab2.txt || exit 1
  done
done
CLIPK_PREFIX_F32_DEEP=3 PREC=fp32s MODE=vit timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06s/prof_3 -o p -- python3 -u tools/lab/vit_contention.py 10 > gpurun_out/r06s/prof_3.log 2>&1
