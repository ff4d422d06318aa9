#!/bin/bash
# GPU tests, then the headline bench under two settings of one env switch (A/B).
# usage: scripts/gpu_ab.sh VAR [outdir]   e.g. scripts/gpu_ab.sh DASH_FUSED_CHAIN
set -e
VAR=${1:?env var}
OUT=${2:-gpurun_out/ab}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gputests.log" 2>&1
env "$VAR=1" timeout -k 10 300 python bench.py --steps 5 --warmup 1 --verify 1 > "$OUT/bench_1.json" 2> "$OUT/bench_1.err"
env "$VAR=0" timeout -k 10 300 python bench.py --steps 5 --warmup 1 --verify 1 > "$OUT/bench_0.json" 2> "$OUT/bench_0.err"
