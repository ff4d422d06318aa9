#!/bin/bash
# Served phase with 8 garbling workers: slots per group x groups, alternating.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06zf}
mkdir -p "$OUT"
for i in 1 2; do
    for cfg in ${CFGS:-16x3 16x4 8x4 24x3}; do
        set -- ${cfg%x*} ${cfg#*x}
        timeout -k 10 300 python bench.py --steps 2 --warmup 1 --batch 8 --phases main,served --served-slots $1 \
            --served-groups $2 > "$OUT/sv_${1}x${2}_$i.json" 2> "$OUT/sv_${1}x${2}_$i.err" || { tail -20 "$OUT/sv_${1}x${2}_$i.err"; exit 1; }
        python3 -c "
import json; r = json.load(open('$OUT/sv_${1}x${2}_$i.json')); s = r['served']
print('slots $1 groups $2', r['served_inf_per_s'], s['pool_wait_s'], s['batch_latency_ms']['p50'], s['verified'])"
    done
done
