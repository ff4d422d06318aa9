#!/bin/bash
# PMC passes over the GPU garbler (one MiniONN GC, mixed-radix rescale, gpu only) -> summary on stdout
set -e
OUT=${1:-gpurun_out/pmcg2}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
RX="k_project|k_mrs_derive|k_draw|k_relu_finish|k_transpose|k_conv"
run() {
  timeout -s KILL 150 rocprofv3 --kernel-trace --kernel-include-regex "$RX" --pmc "$@" --output-format csv -d "$ROOT/$OUT/p$N" -o run -- python3 "$ROOT/scripts/garble_bench.py" --reps 2 --gpu-only > "$ROOT/$OUT/p$N.log" 2>&1
  N=$((N+1))
}
N=0
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
run SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS
run TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum FETCH_SIZE
run WRITE_SIZE TCP_TCC_WRITE_REQ_sum
cd "$ROOT"
python3 -m dash_amd.utils.pmcsum $(find "$OUT" -name "*counter_collection.csv")
rm -rf "$OUT"/p?
