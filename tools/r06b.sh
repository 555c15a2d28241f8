set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
for v in base nosplit mix0; do
  L=""; [ $v != base ] && L=$PWD/build_ab/$v/libclipk.so
  CLIPK_LIB=$L timeout -k 10 200 python -u tools/split_gemm_bench.py $v >> $O/split_gemm.txt 2>>$O/err.txt || exit 1
done
echo done
