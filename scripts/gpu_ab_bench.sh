#!/bin/bash
# A/B of the headline bench on one GPU box (run from the repo root): bench with the defaults, then with the env
# assignments given as arguments (e.g. DASH_RANGE_GUARD=off); prints value / ms per step / batch-1 latencies.
#   gpurun -- 'bash scripts/gpu_ab_bench.sh <tag> [VAR=value ...]'
set -o pipefail
T=${1:-ab}; shift
OUT=gpurun_out/$T
mkdir -p "$OUT"
PH=${PHASES:-main,latency}
timeout -k 10 300 python bench.py --steps "${STEPS:-20}" --warmup 5 --phases "$PH" > "$OUT/a.json" 2> "$OUT/a.err" \
    || { tail -20 "$OUT/a.err"; exit 1; }
if [ $# -gt 0 ]; then
    env "$@" timeout -k 10 300 python bench.py --steps "${STEPS:-20}" --warmup 5 --phases "$PH" > "$OUT/b.json" \
        2> "$OUT/b.err" || { tail -20 "$OUT/b.err"; exit 1; }
fi
for f in a b; do
    [ -s "$OUT/$f.json" ] && python3 -c "
import json
r = json.load(open('$OUT/$f.json'))
print('$f', r['value'], r['ms_per_step'], r.get('latency_b1_ms'), r.get('latency_b1_host_encoded_ms'),
      r.get('served_inf_per_s'), r.get('range_guard'))"
done
exit 0
