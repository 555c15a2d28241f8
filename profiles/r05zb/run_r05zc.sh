# side stream probed for hardware-queue concurrency: vision-schedule tests, then the default bench
set -o pipefail
O=gpurun_out/r05zc; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vision_schedule_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --eval-images 2000 > $O/bench.json 2> $O/bench.err || exit $?
echo ok
