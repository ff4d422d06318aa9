#!/bin/bash
# Custom PMC passes over the headline bench's online kernels (B GCs, one stream, kernel trace only).
#   bash scripts/pmc_custom.sh OUT REGEX BATCH "COUNTERS pass 1" ["COUNTERS pass 2" ...]
# Each quoted counter list is one rocprofv3 run (keep within the per-block limits: 8 SQ, 4 TCC, 4 TCP, 2 TA,
# 2 TD, 2 GRBM); then scripts/pmc_summary.py sums every counter per kernel.
set -e
OUT=$1
RE=$2
B=$3
shift 3
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --batch $B --streams 1 --verify 0 --phases main"
i=0
for CNT in "$@"; do
    i=$((i + 1))
    timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex "$RE" --pmc $CNT \
        --output-format csv -d "$ROOT/$OUT/p$i" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/p$i.log" 2>&1
done
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT" > "$OUT/summary.txt"
for j in $(seq 1 $i); do rm -rf "$OUT/p$j"; done
cat "$OUT/summary.txt"
