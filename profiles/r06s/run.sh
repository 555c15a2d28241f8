# fp32 prefix attention forward with its loads two units ahead (CLIPK_PREFIX_F32_DEEP 1: 2 waves
# per SIMD; 2: 3 waves per SIMD with spills) against one unit ahead (0): the prefix-attention
# tests in every mode, then the fp32s step interleaved, then rocprof per mode
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06s
F='^>>\|Loading\|Use \|amdgpu.ids'
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "attention_prefix" > gpurun_out/r06s/tests.txt 2>&1 || { tail -30 gpurun_out/r06s/tests.txt; exit 1; }
tail -1 gpurun_out/r06s/tests.txt
for i in 1 2; do
  for d in 0 1 2; do
    echo "=== deep $d" >> gpurun_out/r06s/ab.txt
    CLIPK_PREFIX_F32_DEEP=$d PREC=fp32s MODE=vit timeout -k 10 240 python -u tools/lab/vit_contention.py 30 2>&1 | grep -v "$F" >> gpurun_out/r06s/ab.txt || exit 1
  done
done
for d in 0 1 2; do
  CLIPK_PREFIX_F32_DEEP=$d PREC=fp32s MODE=vit timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06s/prof_$d -o p -- python3 -u tools/lab/vit_contention.py 10 > gpurun_out/r06s/prof_$d.log 2>&1 || exit 1
done
