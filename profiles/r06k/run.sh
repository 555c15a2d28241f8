# round 6 final build measured: the whole -m gpu suite, smoke, default bench, rocprof, PMC
set -o pipefail
bash tools/gpu_run.sh r06k tests smoke bench prof pmc
