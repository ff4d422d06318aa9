#!/bin/bash
# PMC counter passes over the headline bench (kernel-trace only; no sys/runtime traces).
set -e
OUT=${1:-gpurun_out/pmc}
B=${2:-8}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d "$ROOT/$OUT/p1" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --batch "$B" --verify 0 > "$ROOT/$OUT/p1.log" 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$ROOT/$OUT/p2" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --batch "$B" --verify 0 > "$ROOT/$OUT/p2.log" 2>&1
