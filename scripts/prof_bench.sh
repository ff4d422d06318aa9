#!/bin/bash
# Kernel-level profile of the headline bench (run on the GPU box from the repo root): main phase only unless
# PHASES is set (AFTER=gg:: adds the timeline after the last garbling kernel: with PHASES=latency, the final
# batch-1 evaluation), B GCs (default 8; the headline config is 160 GCs on 8 streams).
set -e
OUT=${1:-gpurun_out/prof}
B=${2:-8}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --batch "$B" --phases "${PHASES:-main}" ${EXTRA:-} > "$ROOT/$OUT/bench.json" 2> "$ROOT/$OUT/bench.err"
cd "$ROOT"
DB=$(find "$OUT" -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" ${AFTER:+--after "$AFTER"} > "$OUT/summary.txt" 2>&1 || true
