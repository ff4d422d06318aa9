#!/bin/bash
# GPU garbler A/B of two builds on one lease (garble + load per MiniONN GC into evaluator slots, alternating),
# then a kernel trace of each:
#   gpurun -- 'bash scripts/gpu_garble_ab.sh <tag> <tree A> <tree B> [pairs]'
# A tree is a directory holding a built dash_amd/ (e.g. abx/ with the baseline sources, or . for this tree).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=$1 A=$2 B=$3 PAIRS=${4:-2}
OUT=gpurun_out/$T
mkdir -p "$OUT"
for i in $(seq 1 "$PAIRS"); do
    for v in "$A" "$B"; do
        n=$(basename "$(realpath "$v")")
        DASH_PKG_ROOT=$(realpath "$v") timeout -k 10 300 python scripts/garble_bench.py --sink 12 \
            > "$OUT/sink_${n}_$i.json" 2> "$OUT/sink_${n}_$i.err" || { tail -20 "$OUT/sink_${n}_$i.err"; exit 1; }
        echo "$n $(cat "$OUT/sink_${n}_$i.json" | cut -c1-120)"
    done
done
for v in "$A" "$B"; do
    n=$(basename "$(realpath "$v")")
    DASH_PKG_ROOT=$(realpath "$v") timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$n" -o run -- \
        python3 scripts/garble_bench.py --gpu-only --reps 4 > "$OUT/prof_$n.log" 2>&1 || { tail -20 "$OUT/prof_$n.log"; exit 1; }
    db=$(find "$OUT/prof_$n" -name '*.db' | head -1)
    python3 -m dash_amd.utils.profsum "$db" 8 || true
done
