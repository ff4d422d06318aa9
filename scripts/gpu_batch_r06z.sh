#!/bin/bash
# Pipelined steps: streams 4 / 8 / 2 on the main and reference phases, alternating.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06z
mkdir -p "$OUT"
for i in 1 2; do
    for st in 4 8 2; do
        timeout -k 10 400 python bench.py --steps 20 --warmup 5 --phases main,reference --streams $st \
            > "$OUT/mr_s${st}_$i.json" 2> "$OUT/mr_s${st}_$i.err" || { tail -20 "$OUT/mr_s${st}_$i.err"; exit 1; }
        python3 -c "
import json; r = json.load(open('$OUT/mr_s${st}_$i.json')); print('streams $st', r['value'], r['ms_per_step'], r['config']['global_batch'], r['reference_constructions_value'], r['verified_last_timed_step'])"
    done
done
