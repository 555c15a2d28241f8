#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only) for one GEMM shape and for
# the bench's roofline kernel. Usage (on the GPU box, from the repo root): tools/pmc.sh <outdir>
set -e
R=$(pwd)
OUT=$R/${1:-gpurun_out/pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters..., -- cmd
  local name=$1; shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done; shift
  timeout -k 10 300 rocprofv3 --pmc "${ctrs[@]}" --output-format csv -d $OUT/$name -o p -- "$@" > $OUT/$name.log 2>&1
}
for shape in plain dgelu; do
  run ${shape}_sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 $R/tools/one_gemm.py $shape 5
  run ${shape}_fetch FETCH_SIZE -- python3 $R/tools/one_gemm.py $shape 5
  run ${shape}_write WRITE_SIZE -- python3 $R/tools/one_gemm.py $shape 5
  run ${shape}_lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_VALU -- python3 $R/tools/one_gemm.py $shape 5
done
# bench roofline kernel traffic (EPI_DQGELU instantiation only)
run bench_fetch FETCH_SIZE -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof --eval-images 0
run bench_write WRITE_SIZE -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof --eval-images 0
echo pmc done
