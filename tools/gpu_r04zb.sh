# round-4 final pass on the final build: default bench line (as the driver runs it), rocprofv3
# kernel stats of the headline workload, PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes),
# smoke()
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04zb
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra --eval-images 0 > $O/prof.log 2>&1) && \
timeout -k 10 600 bash tools/pmc_bench.sh gpurun_out/r04zb/pmc > $O/pmc.log 2>&1 && \
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
rc=$?
echo exit $rc
exit $rc
