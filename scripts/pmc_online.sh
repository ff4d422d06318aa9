#!/bin/bash
# L1/L2 access-rate and instruction-mix passes over the online evaluation (bench, B GCs, 1 step)
set -e
OUT=${1:-gpurun_out/pmco}
B=${2:-8}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --output-format csv -d "$ROOT/$OUT/a" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --batch "$B" --verify 0 --garble-device 1 > "$ROOT/$OUT/a.log" 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d "$ROOT/$OUT/c" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --batch "$B" --verify 0 > "$ROOT/$OUT/c.log" 2>&1
