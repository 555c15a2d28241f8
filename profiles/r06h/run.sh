# round 6 build measured: headline parity reports, the whole -m gpu suite, smoke, default bench, rocprof, PMC
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -q -s -k "headline_batch8" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_headline_reports.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
bash tools/gpu_run.sh r06h tests smoke bench prof pmc
