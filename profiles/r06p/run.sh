# round 6 final build (split-form epilogue stores by v_fma_mix) measured: the whole -m gpu suite,
# smoke, default bench, rocprof, PMC
set -o pipefail
bash tools/gpu_run.sh r06p tests smoke bench prof pmc
