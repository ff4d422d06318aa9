#!/bin/bash
# Served phase: garbling workers / GPU garbler contexts 4 (default) vs 6 vs 8, alternating.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06zc}
mkdir -p "$OUT"
for i in 1 2; do
    for w in ${WORKERS:-4 6 8}; do
        DASH_GARBLE_WORKERS=$w DASH_GG_CONTEXTS=$w timeout -k 10 300 python bench.py --steps 2 --warmup 1 --batch 8 \
            --phases main,served > "$OUT/sv_w${w}_$i.json" 2> "$OUT/sv_w${w}_$i.err" || { tail -20 "$OUT/sv_w${w}_$i.err"; exit 1; }
        python3 -c "
import json; r = json.load(open('$OUT/sv_w${w}_$i.json')); s = r['served']
print('workers $w', r['served_inf_per_s'], s['pool_wait_s'], s['garble_s_per_gc'], s['batch_latency_ms']['p50'], s['verified'])"
    done
done
