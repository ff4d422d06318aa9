#!/bin/bash
# Stream-group sweep of the headline bench at B=24 (one bench run per setting).
set -e
OUT=${1:-gpurun_out/sweep}
mkdir -p "$OUT"
for s in ${STREAMS:-2 3 6 8 12}; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --verify 0 --streams $s > "$OUT/s$s.json" 2> "$OUT/s$s.err"
done
