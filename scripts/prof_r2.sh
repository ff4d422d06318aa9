#!/bin/bash
# Kernel trace of the headline bench at its default config, then PMC passes (one
# counter block set per run) at B=8 on one stream so kernels do not overlap.
# Run on the GPU box: scripts/prof_r2.sh [outdir]
set -e
OUT=${1:-gpurun_out/prof}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/kt" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --verify 0 > "$ROOT/$OUT/bench.json" 2> "$ROOT/$OUT/bench.err"
cd "$ROOT"
DB=$(find "$OUT/kt" -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" > "$OUT/summary.txt" 2>&1 || true
cd /tmp
B8="--steps 1 --warmup 0 --verify 0 --batch 8 --streams 1"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d "$ROOT/$OUT/p1" -o run -- python3 "$ROOT/bench.py" $B8 > "$ROOT/$OUT/p1.log" 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$ROOT/$OUT/p2" -o run -- python3 "$ROOT/bench.py" $B8 > "$ROOT/$OUT/p2.log" 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR --output-format csv -d "$ROOT/$OUT/p3" -o run -- python3 "$ROOT/bench.py" $B8 > "$ROOT/$OUT/p3.log" 2>&1
cd "$ROOT"
python3 -m dash_amd.utils.pmcsum $(find "$OUT/p1" "$OUT/p2" "$OUT/p3" -name "*counter_collection.csv") > "$OUT/pmc.txt" 2>&1 || true
