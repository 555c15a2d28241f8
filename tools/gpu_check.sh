#!/bin/bash
# quick GPU check after a change: the -m gpu suite (or the files given) under one time limit
R=$(pwd)
mkdir -p gpurun_out
TAG=${TAG:-chk}
timeout -k 10 600 python -u -m pytest ${@:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
tail -n 3 gpurun_out/gpu_tests_$TAG.log
exit $rc
