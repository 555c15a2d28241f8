# the 125-class proxy inside the default bench run, with and without gc.collect + gc.freeze
set -o pipefail
O=gpurun_out/r05z; mkdir -p $O
for g in "" 1; do
  BENCH_GC=$g timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --eval-images 2000 > $O/bench_gc$g.json 2> $O/bench_gc$g.err || exit $?
done
echo ok
