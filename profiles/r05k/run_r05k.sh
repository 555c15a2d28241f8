set -o pipefail
O=gpurun_out/r05k; mkdir -p $O
for c in 1000 250 125; do
  timeout -k 10 240 python -u bench.py --batch 1 --classes $c --steps 50 --warmup 5 --no-extra --no-cpu-baseline --eval-images 100 > $O/b1_c$c.json 2> $O/b1_c$c.err || exit $?
done
echo ok
