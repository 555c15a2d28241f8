#!/bin/bash
# The one maintained GPU-box runner (replaces the per-lease gpu_r0*.sh scripts of rounds 2-4).
# Usage, from the repo root on the GPU box:  bash tools/gpu_run.sh <tag> <stage> [<stage> ...]
# Stages (run in the order given; each under its own time limit; outputs in gpurun_out/<tag>/):
#   tests   the whole `pytest -m gpu` suite            -> gpu_tests.txt
#   smoke   __graft_entry__.smoke()                     -> smoke.txt
#   bench   the default `python bench.py` line          -> bench.json (+ bench.err)
#   quick   bench.py --no-extra (headline line only)    -> bench_quick.json
#   prof    rocprofv3 --kernel-trace --stats of the headline train step alone -> prof/
#   pmc     FETCH_SIZE / WRITE_SIZE passes (tools/pmc_bench.sh)               -> pmc/
# A failing test run (exit 1) lets the later stages run; any other failure (a fault, an abort, a
# time limit) ends the script there.
set -o pipefail
R=$(pwd)
TAG=${1:?tag}
shift
O=$R/gpurun_out/$TAG
mkdir -p $O
stage() {
  local name=$1 rc
  shift
  echo "[$(date +%T)] $name" >> $O/stages.log
  "$@"
  rc=$?
  echo "[$(date +%T)] $name exit $rc" >> $O/stages.log
  if [ $rc -ne 0 ] && ! { [ $name = tests ] && [ $rc -eq 1 ]; }; then
    echo "stage $name failed ($rc): stopping"
    exit $rc
  fi
}
for s in "$@"; do
  case $s in
    tests) stage tests timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
             -p no:cacheprovider > $O/gpu_tests.txt 2>&1 ;;
    smoke) stage smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 ;;
    bench) stage bench timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err ;;
    quick) stage quick timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline \
             > $O/bench_quick.json 2> $O/bench_quick.err ;;
    prof) stage prof bash -c "cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
             --output-format csv -d $O/prof -o p -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline \
             --no-extra --eval-images 0 > $O/prof.log 2>&1" ;;
    pmc) stage pmc timeout -k 10 600 bash tools/pmc_bench.sh gpurun_out/$TAG/pmc > $O/pmc.log 2>&1 ;;
    *) echo "unknown stage $s"; exit 2 ;;
  esac
done
echo "all stages done"
