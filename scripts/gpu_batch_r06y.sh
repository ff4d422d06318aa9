#!/bin/bash
# Headline with pipelined steps: stream (group) count A/B, alternating, main phase.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06y
mkdir -p "$OUT"
for i in 1 2; do
    for st in 8 16 4 10; do
        timeout -k 10 400 python bench.py --steps 20 --warmup 5 --phases main --streams $st \
            > "$OUT/main_s${st}_$i.json" 2> "$OUT/main_s${st}_$i.err" || { tail -20 "$OUT/main_s${st}_$i.err"; exit 1; }
        python3 -c "
import json; r = json.load(open('$OUT/main_s${st}_$i.json')); print('streams $st', r['value'], r['ms_per_step'], r['config']['global_batch'], r['verified_last_timed_step'])"
    done
done
for i in 1 2; do
    for o in index completion; do
        DASH_BENCH_ORDER=$o timeout -k 10 400 python bench.py --steps 20 --warmup 5 --phases main \
            > "$OUT/main_o${o}_$i.json" 2> "$OUT/main_o${o}_$i.err" || { tail -20 "$OUT/main_o${o}_$i.err"; exit 1; }
        python3 -c "
import json; r = json.load(open('$OUT/main_o${o}_$i.json')); print('order $o', r['value'], r['ms_per_step'], r['verified_last_timed_step'])"
    done
done
