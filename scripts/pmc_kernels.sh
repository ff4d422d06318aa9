#!/bin/bash
# PMC counter passes over selected online kernels of the headline bench (B GCs, one stream, kernel trace only).
#   [STREAMS=8] bash scripts/pmc_kernels.sh OUT [REGEX] [BATCH]
# Two passes (the SQ block holds 8 counters per run), then a per-kernel summary: counters summed over
# dispatches, derived ratios (LDS bank-conflict %, MFMA busy %, waiting %) and GPU ms per kernel.
set -e
OUT=${1:-gpurun_out/pmc}
RE=${2:-k_mrs_chain|k_rescale_mrs_out_hash|k_relu_mult|k_conv_img2}
B=${3:-24}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --batch $B --streams ${STREAMS:-1} --verify 0 --phases main ${EXTRA:-}"
timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex "$RE" \
    --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES \
    --output-format csv -d "$ROOT/$OUT/a" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/a.log" 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex "$RE" \
    --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM \
    --output-format csv -d "$ROOT/$OUT/b" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/b.log" 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex "$RE" --pmc FETCH_SIZE \
    --output-format csv -d "$ROOT/$OUT/c" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/c.log" 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex "$RE" --pmc WRITE_SIZE \
    --output-format csv -d "$ROOT/$OUT/d" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/d.log" 2>&1
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT" > "$OUT/summary.txt"
rm -rf "$OUT/a" "$OUT/b" "$OUT/c" "$OUT/d"
cat "$OUT/summary.txt"
