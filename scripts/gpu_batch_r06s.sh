#!/bin/bash
# Coop pad in k_rescale_relu_out_q: GPU tests, batch-1 latency of this tree against aby/, and a batch-1 timeline.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06s
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.txt" 2>&1 \
    || { tail -40 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
for i in 1 2; do
    for t in aby .; do
        n=$(basename "$(realpath "$t")")
        (cd "$t" && timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch 8 --phases main,latency --latency-gcs 8) \
            > "$OUT/lat_${n}_$i.json" 2> "$OUT/lat_${n}_$i.err" || { tail -20 "$OUT/lat_${n}_$i.err"; exit 1; }
        python3 -c "
import json; r = json.load(open('$OUT/lat_${n}_$i.json')); print('$n', r['latency_b1_ms'], r['latency_b1']['min_ms'], r['latency_b1']['verified'])"
    done
done
PHASES=latency AFTER=gg:: EXTRA="--latency-gcs 4" bash scripts/prof_bench.sh gpurun_out/r06s_b1 4 && tail -45 gpurun_out/r06s_b1/summary.txt
