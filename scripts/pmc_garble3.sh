#!/bin/bash
# PMC roofline of the GPU garbler's kernels (MiniONN GC, flagship constructions, gpu only) -> summary on stdout
set -e
OUT=${1:-gpurun_out/pmcg3}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
RX="k_hash_iu|k_hash_jobs|k_bank|k_emit|k_draw|k_mrs_derive|k_relu_finish|k_conv|k_chunk_res|k_bin_keys"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --kernel-include-regex "$RX" -d "$ROOT/$OUT/kt" -o run -- python3 "$ROOT/scripts/garble_bench.py" --reps 4 --gpu-only > "$ROOT/$OUT/kt.log" 2>&1
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
DB=$(find $OUT/kt -name "*.db" | head -n 1)
if [ -n "$DB" ]; then python3 -m dash_amd.utils.profsum "$DB" 30 || true; else find $OUT/kt -name "*stats*" -exec cat {} \; ; fi
python3 -m dash_amd.utils.pmcsum $(find "$OUT" -name "*counter_collection.csv")
rm -rf "$OUT"/p? "$OUT"/kt
