#!/bin/bash
# Batch-1 latency recheck: this tree twice and the round-start tree aby/ once, same lease.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zk
mkdir -p "$OUT"
for t in . aby .; do
    n=$(basename "$(realpath "$t")")_$RANDOM
    (cd "$t" && timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch 8 --phases main,latency --latency-gcs 8) \
        > "$OUT/lat_$n.json" 2> "$OUT/lat_$n.err" || { tail -20 "$OUT/lat_$n.err"; exit 1; }
    python3 -c "
import json; r = json.load(open('$OUT/lat_$n.json')); print('$n', r['latency_b1_ms'], r['latency_b1']['min_ms'], r.get('latency_b1_host_encoded_ms'))"
done
