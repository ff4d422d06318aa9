#!/bin/bash
# Conv PMC of the online step (k_conv_img2, B GCs, one stream): the GPU garbler's conv dispatches (it reuses the
# kernel) are dropped by PMC_AFTER=gg:: in the summary. Passes: the SQ set, then MFMA busy + int8 MOPS.
#   bash scripts/pmc_conv.sh OUT [BATCH]
set -e
OUT=${1:-gpurun_out/pmc_conv}
B=${2:-24}
ROOT=$(pwd)
RE='k_conv_img2|gg::k_emit'
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --batch $B --streams 1 --verify 0 --phases main"
timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex "$RE" \
    --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    --output-format csv -d "$ROOT/$OUT/a" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/a.log" 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex "$RE" \
    --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
    --output-format csv -d "$ROOT/$OUT/b" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/b.log" 2>&1
cd "$ROOT"
PMC_AFTER=gg:: python3 scripts/pmc_summary.py "$OUT" > "$OUT/summary.txt"
rm -rf "$OUT/a" "$OUT/b"
cat "$OUT/summary.txt"
