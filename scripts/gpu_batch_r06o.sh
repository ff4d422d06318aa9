#!/bin/bash
# Round-6 combined GPU pass: GPU tests, online A/B of three trees (abx: round-6 baseline, aby: p = 2 digit
# window in the rescale output kernel, .: plus compile-time whole-chunk digit loops), garbler knob A/B, served
# slots A/B. Each step under its own time limit; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06o
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
for i in 1 2; do
    for v in abx aby .; do
        n=$(basename "$(realpath "$v")")
        timeout -k 10 300 python scripts/ab_online.py --root "$v" --batch 24 --steps 5 --relu joint \
            > "$OUT/online_${n}_$i.json" 2> "$OUT/online_${n}_$i.err" || { tail -20 "$OUT/online_${n}_$i.err"; exit 1; }
        echo "$n $(head -1 "$OUT/online_${n}_$i.json" | cut -c1-300)"
    done
done
timeout -k 10 500 bash scripts/gpu_garble_env_ab.sh r06o_garble - DASH_GG_AES_COPIES=16 DASH_GG_DRAW_BLOCKS=512 || exit 1
for s in 16 32; do
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --phases main,served --served-slots $s \
        > "$OUT/served_$s.json" 2> "$OUT/served_$s.err" || { tail -20 "$OUT/served_$s.err"; exit 1; }
    python3 -c "
import json; r = json.load(open('$OUT/served_$s.json')); print('slots $s', r['value'], r['served_inf_per_s'], r['served']['batch_latency_ms'], r['served']['pool_wait_s'])"
done
