#!/bin/bash
# One GPU-box validation pass (run from the repo root on the box):
#   gpurun -- 'bash scripts/gpu_round.sh <tag>'
# Steps, each under its own time limit and stopping at the first failure:
#   GPU tests -> smoke -> per-model garbling times -> headline bench -> two-party bench.
# Skip steps with SKIP_TESTS=1 / SKIP_GARBLE=1 / SKIP_BENCH=1 / SKIP_TP=1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:-round}
OUT=gpurun_out/$T
mkdir -p "$OUT"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
    tail -1 "$OUT/gpu_tests.log"
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { tail -20 "$OUT/smoke.log"; exit 1; }
    tail -1 "$OUT/smoke.log"
fi
if [ "${SKIP_GARBLE:-0}" != 1 ]; then
    timeout -k 10 300 python -u scripts/garble_models.py 5 > "$OUT/garble_models.jsonl" 2> "$OUT/garble_models.err" \
        || { tail -20 "$OUT/garble_models.err"; exit 1; }
    cat "$OUT/garble_models.jsonl"
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
    timeout -k 10 900 python bench.py --steps "${STEPS:-20}" --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
        || { tail -20 "$OUT/bench.err"; exit 1; }
    cat "$OUT/bench.json"
fi
if [ "${SKIP_TP:-0}" != 1 ]; then
    timeout -k 10 600 python -u benchmarks/two_party.py \
        --models "${TP_MODELS:-MODEL_A/SIMPLE,MODEL_F_MINIONN_POOL_REPL/DASH,MODEL_F_MINIONN_POOL_REPL/OPT}" \
        --batch 4 --rounds 3 --out "$OUT/two_party.jsonl" > "$OUT/two_party.log" 2>&1 \
        || { tail -30 "$OUT/two_party.log"; exit 1; }
    cat "$OUT/two_party.jsonl"
fi
