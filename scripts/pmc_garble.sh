#!/bin/bash
# PMC passes over the GPU garbler (one MiniONN GC, gpu only)
set -e
OUT=${1:-gpurun_out/pmcg}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$ROOT/$OUT/a" -o run -- python3 "$ROOT/scripts/garble_bench.py" --reps 1 --gpu-only > "$ROOT/$OUT/a.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT --output-format csv -d "$ROOT/$OUT/b" -o run -- python3 "$ROOT/scripts/garble_bench.py" --reps 1 --gpu-only > "$ROOT/$OUT/b.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum FETCH_SIZE --output-format csv -d "$ROOT/$OUT/c" -o run -- python3 "$ROOT/scripts/garble_bench.py" --reps 1 --gpu-only > "$ROOT/$OUT/c.log" 2>&1
