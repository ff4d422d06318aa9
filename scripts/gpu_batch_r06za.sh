#!/bin/bash
# Reference-constructions phase: 1 / 2 / 3 groups (--ref-streams), alternating; main phase at the new default.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06za
mkdir -p "$OUT"
for i in 1 2; do
    for rs in 2 1 3; do
        timeout -k 10 400 python bench.py --steps 20 --warmup 5 --phases main,reference --ref-streams $rs \
            > "$OUT/r_s${rs}_$i.json" 2> "$OUT/r_s${rs}_$i.err" || { tail -20 "$OUT/r_s${rs}_$i.err"; exit 1; }
        python3 -c "
import json; r = json.load(open('$OUT/r_s${rs}_$i.json')); c = r['reference_constructions']
print('ref streams $rs', c['value'], c['gcs_per_gpu'], c['streams'], c['verified_last_timed_step'], 'main', r['value'], r['config']['streams'])"
    done
done
