#!/bin/bash
# The other BASELINE configurations through the headline bench (run on the GPU box from the repo root):
# main phase (as many GCs as HBM holds, capped at 256) + batch-1 latency, every run verified against the
# plaintext model. One JSON record per model in OUT/models.jsonl.
set -o pipefail
OUT=${1:-gpurun_out/models}
mkdir -p "$OUT"
: > "$OUT/models.jsonl"
for mc in MODEL_F_GNNP_POOL_REPL:DASH MODEL_F_MINIONN_POOL_REPL:REDASH_OPT MODEL_F_MINIONN_POOL_REPL:REDASH_CPM \
          LENET5:DASH MODEL_A:DASH VGG16:DASH RESNET18:DASH; do
    m=${mc%%:*} c=${mc##*:}
    timeout -k 10 420 python bench.py --model "$m" --config "$c" --steps "${STEPS:-10}" --warmup 2 \
        --phases main,latency --latency-gcs 4 > "$OUT/$m.$c.json" 2> "$OUT/$m.$c.err" \
        || { echo "$m $c failed"; tail -15 "$OUT/$m.$c.err"; exit 1; }
    cat "$OUT/$m.$c.json" >> "$OUT/models.jsonl"
    python3 -c "
import json; r = json.load(open('$OUT/$m.$c.json'))
print('$m', '$c', r['value'], r['ms_per_inference'], r['config']['gcs_per_gpu'], r['offline']['table_gb_per_gc'],
      r.get('latency_b1_ms'), r['config']['encoding'], r['verified_vs_plaintext'])"
done
