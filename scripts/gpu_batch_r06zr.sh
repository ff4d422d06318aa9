#!/bin/bash
# Main phase: groups x hardware queues (GPU_MAX_HW_QUEUES; the box default is 4), alternating.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zr
mkdir -p "$OUT"
for i in 1 2; do
    for cfg in 3x4 4x8 6x8 3x8; do
        st=${cfg%x*} q=${cfg#*x}
        GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python bench.py --steps 20 --warmup 5 --phases main --streams $st \
            > "$OUT/main_${cfg}_$i.json" 2> "$OUT/main_${cfg}_$i.err" || { tail -20 "$OUT/main_${cfg}_$i.err"; exit 1; }
        python3 -c "
import json; r = json.load(open('$OUT/main_${cfg}_$i.json')); print('groups x queues $cfg', r['value'], r['ms_per_step'], r['config']['global_batch'], r['verified_last_timed_step'])"
    done
done
