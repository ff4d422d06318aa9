#!/bin/bash
# Kernel trace + PMC passes of the headline bench at its default config (run on the GPU box).
set -e
OUT=${1:-gpurun_out/prof24}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/kt" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --verify 0 > "$ROOT/$OUT/bench.json" 2> "$ROOT/$OUT/bench.err"
cd "$ROOT"
DB=$(find "$OUT/kt" -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" > "$OUT/summary.txt" 2>&1 || true
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d "$ROOT/$OUT/p1" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --verify 0 --batch 8 --streams 1 > "$ROOT/$OUT/p1.log" 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$ROOT/$OUT/p2" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --verify 0 --batch 8 --streams 1 > "$ROOT/$OUT/p2.log" 2>&1
