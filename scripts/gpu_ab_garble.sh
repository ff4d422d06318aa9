#!/bin/bash
# GPU-garbler timing for the main tree and every built ab/<variant>, back to back (GPU only, 3 reps).
set -e
OUT=${1:-gpurun_out/abg}
mkdir -p "$OUT"
timeout -k 10 200 python scripts/garble_bench.py --reps 3 --gpu-only > "$OUT/main.json" 2> "$OUT/main.err"
for d in ab/*/; do
  n=$(basename "$d")
  timeout -k 10 200 python "$d/scripts/garble_bench.py" --reps 3 --gpu-only > "$OUT/$n.json" 2> "$OUT/$n.err"
done
