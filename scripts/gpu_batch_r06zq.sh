#!/bin/bash
# k_encode_in rows per block: GPU tests, a headline kernel trace, then the group-count A/B of the main phase.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06zq
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.txt" 2>&1 \
    || { tail -40 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
bash scripts/prof_bench.sh gpurun_out/r06zq_prof 164 && grep -E "k_encode_in|TOTAL" gpurun_out/r06zq_prof/summary.txt || exit 1
bash scripts/gpu_batch_r06zp.sh
