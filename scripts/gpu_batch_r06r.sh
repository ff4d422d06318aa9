#!/bin/bash
# Quad-cooperative ChaCha pads in k_mrs_chain_q: GPU tests of this tree, then batch-1 latency and the 24-GC online
# step of this tree (.) against the baseline tree aby/, alternating on one lease.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06r
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
bash scripts/gpu_online_ab.sh r06r_online aby . 2
