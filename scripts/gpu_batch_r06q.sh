#!/bin/bash
# Fused k_emit (DASH_GG_FUSED): byte identity against the host garbler, garbler A/B fused vs staged, guard
# stream-priority A/B of the batch-1 latency, then the other model configurations.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06q
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_two_party.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -3 "$OUT/tests.txt"
bash scripts/gpu_garble_env_ab.sh r06q_fuse "DASH_GG_FUSED=0" "-" || exit 1
for pr in 2 0 2 0; do
    DASH_GUARD_PRIO=$pr timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch 8 --phases main,latency \
        --latency-gcs 8 > "$OUT/lat_p$pr.json" 2> "$OUT/lat_p$pr.err" || { tail -20 "$OUT/lat_p$pr.err"; exit 1; }
    python3 -c "
import json; r = json.load(open('$OUT/lat_p$pr.json')); print('prio $pr', r['latency_b1_ms'], r['latency_b1'])"
done
STEPS=5 bash scripts/gpu_models.sh gpurun_out/models
