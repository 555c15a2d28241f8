# round-4: rocprofv3 kernel stats of the PREC fp32s workload on the final build (the fp32s line's
# roofline kernel: the N = 512 input-grad split GEMMs)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04zc
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 $R/bench.py --prec fp32s --steps 10 --warmup 3 --no-cpu-baseline --no-extra --no-configs --eval-images 0 > $O/prof.log 2>&1)
rc=$?
echo exit $rc
exit $rc
