#!/bin/bash
# Garbler copy trace, the other model configurations, and a guard stream-priority A/B of the batch-1 latency.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06p
mkdir -p "$OUT"
bash scripts/prof_garble_copies.sh gpurun_out/gcopy || exit 1
for pr in 2 0 2 0; do
    DASH_GUARD_PRIO=$pr timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch 8 --phases main,latency \
        --latency-gcs 8 > "$OUT/lat_p$pr.json" 2> "$OUT/lat_p$pr.err" || { tail -20 "$OUT/lat_p$pr.err"; exit 1; }
    python3 -c "
import json; r = json.load(open('$OUT/lat_p$pr.json')); print('prio $pr', r['latency_b1_ms'], r['latency_b1'])"
done
bash scripts/gpu_models.sh gpurun_out/models
