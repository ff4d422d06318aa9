#!/bin/bash
# Batch-1 latency A/B of one environment knob, alternating runs on one lease:
#   gpurun -- 'bash scripts/gpu_b1_ab.sh <tag> <VAR> <a> <b> [pairs]'
# Each run: the main phase (short) plus the latency phase (--latency-gcs fresh GCs one by one).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=$1 VAR=$2 A=$3 B=$4 PAIRS=${5:-2}
OUT=gpurun_out/$T
mkdir -p "$OUT"
for i in $(seq 1 "$PAIRS"); do
    for v in "$A" "$B"; do
        env "$VAR=$v" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch 16 --phases latency --latency-gcs 16 \
            > "$OUT/${VAR}_${v}_$i.json" 2> "$OUT/${VAR}_${v}_$i.err" || { tail -20 "$OUT/${VAR}_${v}_$i.err"; exit 1; }
        python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d.get('latency_b1_ms'), d['value'])" \
            "$OUT/${VAR}_${v}_$i.json" "$VAR=$v"
    done
done
