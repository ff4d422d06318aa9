#!/bin/bash
# GPU garbler A/B: key hashes / bank payloads (DASH_GG_KEYS = 0 round-3 per-lane forms, 1 bank rows from the
# offsets' multiple rows, 2 + uniform-i key hashes): garble + load time per GC into evaluator slots, and a kernel
# trace per mode
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r4keys}
ROOT=$(pwd)
OUT=gpurun_out/$T
mkdir -p $OUT
for m in ${MODES:-2 0 1}; do
  DASH_GG_KEYS=$m timeout -k 10 180 python scripts/garble_bench.py --sink 24 > $OUT/sink_$m.json 2> $OUT/sink_$m.err || { tail -20 $OUT/sink_$m.err; exit 1; }
  echo "keys=$m $(cat $OUT/sink_$m.json)"
done
cd /tmp
for m in ${KT_MODES:-2 0}; do
  DASH_GG_KEYS=$m timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/kt$m" -o run -- python3 "$ROOT/scripts/garble_bench.py" --reps 4 --gpu-only > "$ROOT/$OUT/kt$m.log" 2>&1 || { tail -5 "$ROOT/$OUT/kt$m.log"; exit 1; }
  DB=$(find "$ROOT/$OUT/kt$m" -name "*.db" | head -n 1)
  (cd "$ROOT" && python3 -m dash_amd.utils.profsum "$DB" 16 > "$OUT/kt_summary_$m.txt" 2>&1) || true
  rm -rf "$ROOT/$OUT/kt$m"
  echo "== kernel trace keys=$m (4 GCs)"; head -18 "$ROOT/$OUT/kt_summary_$m.txt"
done
