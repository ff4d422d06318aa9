#!/bin/bash
# Main phase with pipelined steps: 3 / 4 / 5 / 6 groups, alternating.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zp
mkdir -p "$OUT"
for i in 1 2; do
    for st in 4 3 5 6; do
        timeout -k 10 400 python bench.py --steps 20 --warmup 5 --phases main --streams $st \
            > "$OUT/main_s${st}_$i.json" 2> "$OUT/main_s${st}_$i.err" || { tail -20 "$OUT/main_s${st}_$i.err"; exit 1; }
        python3 -c "
import json; r = json.load(open('$OUT/main_s${st}_$i.json')); print('streams $st', r['value'], r['ms_per_step'], r['config']['global_batch'], r['verified_last_timed_step'])"
    done
done
