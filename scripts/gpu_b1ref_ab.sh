#!/bin/bash
# Batch-1 latency of the reference's constructions (latency_ref phase), A/B of one environment knob, alternating:
#   gpurun -- 'bash scripts/gpu_b1ref_ab.sh <tag> <VAR> <a> <b> [pairs]'
set -o pipefail
export TMPDIR=/tmp
T=$1 VAR=$2 A=$3 B=$4 PAIRS=${5:-2}
OUT=gpurun_out/$T
mkdir -p "$OUT"
for i in $(seq 1 "$PAIRS"); do
    for v in "$A" "$B"; do
        env "$VAR=$v" timeout -k 10 300 python bench.py --steps 1 --warmup 0 --batch 1 --phases latency_ref \
            --latency-gcs 6 > "$OUT/${VAR}_${v}_$i.json" 2> "$OUT/${VAR}_${v}_$i.err" || { tail -20 "$OUT/${VAR}_${v}_$i.err"; exit 1; }
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d.get('latency_b1_reference_ms'), d.get('latency_b1_reference', {}).get('verified'))" \
            "$OUT/${VAR}_${v}_$i.json" "$VAR=$v"
    done
done
