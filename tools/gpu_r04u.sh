# round-4 GPU pass u: the batch-1 step under the kernel tracer (tools/trace_steps.py summary)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r04u_b1 -o p -- python3 $R/tools/cpu_issue_probe.py --batches 1 --steps 20 > $R/gpurun_out/r04u_b1.log 2>&1 && \
cd $R && python3 tools/trace_steps.py gpurun_out/r04u_b1/p_kernel_trace.csv --skip 3 --steps 10 > gpurun_out/r04u_b1_trace.txt 2>&1
rc=$?
echo exit $rc
exit $rc
