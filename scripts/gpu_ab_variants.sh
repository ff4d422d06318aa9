#!/bin/bash
# Headline bench for the main tree and every built ab/<variant> (scripts/ab_variant.sh), back to back.
set -e
OUT=${1:-gpurun_out/abv}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --verify 1 > "$OUT/main.json" 2> "$OUT/main.err"
for d in ab/*/; do
  n=$(basename "$d")
  timeout -k 10 300 python "$d/bench.py" --steps 5 --warmup 1 --verify 1 > "$OUT/$n.json" 2> "$OUT/$n.err"
done
