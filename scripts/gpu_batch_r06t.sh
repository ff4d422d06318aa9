#!/bin/bash
# Batched AES image fill + coop pad in k_rescale_relu_out_q: GPU tests, then batch-1 latency (flagship and the
# reference's constructions) of this tree against aby/, alternating on one lease.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06t
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.txt" 2>&1 \
    || { tail -40 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
for i in 1 2; do
    for t in aby .; do
        n=$(basename "$(realpath "$t")")
        (cd "$t" && timeout -k 10 400 python bench.py --steps 3 --warmup 1 --batch 8 --phases main,latency,latency_ref \
            --latency-gcs 6) > "$OUT/lat_${n}_$i.json" 2> "$OUT/lat_${n}_$i.err" || { tail -20 "$OUT/lat_${n}_$i.err"; exit 1; }
        python3 -c "
import json; r = json.load(open('$OUT/lat_${n}_$i.json'))
print('$n', r['latency_b1_ms'], r['latency_b1']['min_ms'], r.get('latency_b1_reference_ms'), r.get('latency_b1_host_encoded_ms'))"
    done
done
bash scripts/gpu_b1_ab.sh r06t_rro DASH_RRO_QUAD 1 2 2 || exit 1
bash scripts/gpu_b1_ab.sh r06t_mq DASH_MRS_QUAD 1 0 1 || exit 1
