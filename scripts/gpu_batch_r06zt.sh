#!/bin/bash
# k_encode_in per (slot, residue): GPU tests, headline kernel trace, main-phase bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zt
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.txt" 2>&1 \
    || { tail -40 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
bash scripts/prof_bench.sh gpurun_out/r06zt_prof 165 && grep -E "k_encode_in|TOTAL" gpurun_out/r06zt_prof/summary.txt || exit 1
for i in 1 2; do
    timeout -k 10 400 python bench.py --steps 20 --warmup 5 --phases main,latency > "$OUT/main_$i.json" 2> "$OUT/main_$i.err" \
        || { tail -20 "$OUT/main_$i.err"; exit 1; }
    python3 -c "
import json; r = json.load(open('$OUT/main_$i.json')); print('main', r['value'], r['ms_per_step'], r['latency_b1_ms'], r['verified_last_timed_step'])"
done
