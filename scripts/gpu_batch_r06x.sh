#!/bin/bash
# Headline A/B: groups pipelined across steps (--pipeline 1) against step by step (0), alternating, main phase.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06x
mkdir -p "$OUT"
for i in 1 2; do
    for p in 0 1; do
        timeout -k 10 400 python bench.py --steps 20 --warmup 5 --phases main --pipeline $p \
            > "$OUT/main_p${p}_$i.json" 2> "$OUT/main_p${p}_$i.err" || { tail -20 "$OUT/main_p${p}_$i.err"; exit 1; }
        python3 -c "
import json; r = json.load(open('$OUT/main_p${p}_$i.json')); print('pipeline $p', r['value'], r['ms_per_step'], r['verified_vs_plaintext'], r['verified_last_timed_step'])"
    done
done
