#!/bin/bash
# Online A/B of two package trees (24 MiniONN GCs, one stream, per-op-kind GPU times), alternating on one lease:
#   gpurun -- 'bash scripts/gpu_online_ab.sh <tag> <tree A> <tree B> [pairs]'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=$1 A=$2 B=$3 PAIRS=${4:-2}
OUT=gpurun_out/$T
mkdir -p "$OUT"
for i in $(seq 1 "$PAIRS"); do
    for v in "$A" "$B"; do
        n=$(basename "$(realpath "$v")")
        timeout -k 10 300 python scripts/ab_online.py --root "$v" --batch 24 --steps 5 --relu joint ${DETAIL:+--detail} \
            > "$OUT/online_${n}_$i.json" 2> "$OUT/online_${n}_$i.err" || { tail -20 "$OUT/online_${n}_$i.err"; exit 1; }
        echo "$n $(head -1 "$OUT/online_${n}_$i.json")"
    done
done
