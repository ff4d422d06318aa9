#!/bin/bash
# HBM fetch bytes per kernel over the headline bench (one TCC counter set per run).
set -e
OUT=${1:-gpurun_out/pmcf}
B=${2:-24}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$ROOT/$OUT/f" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --batch "$B" --verify 0 > "$ROOT/$OUT/f.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$ROOT/$OUT/s" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --batch "$B" --verify 0 > "$ROOT/$OUT/s.log" 2>&1
cd "$ROOT" && python3 -m dash_amd.utils.pmcsum $OUT/f/run_counter_collection.csv $OUT/s/run_counter_collection.csv > $OUT/summary.txt
