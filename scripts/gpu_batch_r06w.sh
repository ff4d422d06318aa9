#!/bin/bash
# 16-component chunks in k_rescale_update_approx on latency-bound launches: GPU tests, then the reference
# constructions' batch-1 latency with DASH_UA_SMALL=1 / 0.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06w
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.txt" 2>&1 \
    || { tail -40 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
bash scripts/gpu_b1ref_ab.sh r06w_ua DASH_UA_SMALL 1 0 2
