#!/bin/bash
# Round-6 combined GPU pass (one lease): GPU tests, online A/B (baseline tree abx vs this tree), garbler knob A/B,
# served slots A/B. Each step under its own time limit; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06n
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 600 bash scripts/gpu_online_ab.sh r06n_online abx . 2 || exit 1
timeout -k 10 500 bash scripts/gpu_garble_env_ab.sh r06n_garble - DASH_GG_AES_COPIES=16 DASH_GG_DRAW_BLOCKS=512 || exit 1
for s in 16 32; do
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --phases main,served --served-slots $s \
        > "$OUT/served_$s.json" 2> "$OUT/served_$s.err" || { tail -20 "$OUT/served_$s.err"; exit 1; }
    python3 -c "
import json; r = json.load(open('$OUT/served_$s.json')); print('slots $s', r['served_inf_per_s'], r['served']['batch_latency_ms'], r['served']['pool_wait_s'])"
done
