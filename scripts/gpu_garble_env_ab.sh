#!/bin/bash
# GPU garbler A/B of runtime knobs on one lease: garble + load per MiniONN GC into evaluator slots
# (garble_bench.py --sink 12) with each env setting, alternating, then a kernel trace of each.
#   gpurun -- 'bash scripts/gpu_garble_env_ab.sh <tag> "VAR=a" "VAR=b" ...'   ("-" = defaults)
set -o pipefail
T=$1; shift
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for rep in 1 2; do
    for cfg in "$@"; do
        e=(); [ "$cfg" != "-" ] && e=($cfg)
        env "${e[@]}" timeout -k 10 300 python scripts/garble_bench.py --sink 12 > "$OUT/s_${rep}_$i.json" 2> "$OUT/s_${rep}_$i.err" \
            || { tail -20 "$OUT/s_${rep}_$i.err"; exit 1; }
        echo "[$cfg] $(cut -c1-110 "$OUT/s_${rep}_$i.json")"
        i=$((i + 1))
    done
done
j=0
for cfg in "$@"; do
    e=(); [ "$cfg" != "-" ] && e=($cfg)
    for kv in "${e[@]}"; do export "$kv"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$j" -o run -- python3 scripts/garble_bench.py --gpu-only --reps 4 \
        > "$OUT/prof_$j.log" 2>&1 || { tail -20 "$OUT/prof_$j.log"; exit 1; }
    for kv in "${e[@]}"; do unset "${kv%%=*}"; done
    echo "[$cfg]"
    python3 -m dash_amd.utils.profsum "$(find "$OUT/prof_$j" -name '*.db' | head -1)" 6 || true
    j=$((j + 1))
done
