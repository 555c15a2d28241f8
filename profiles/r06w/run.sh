# round 6 final build (96-row tiles for one-round grids, bench grad_allreduce field at N > 1):
# the whole -m gpu suite, smoke, default bench, rocprof, PMC
set -o pipefail
bash tools/gpu_run.sh r06w tests smoke bench prof pmc
