#!/bin/bash
# PMC of the reference constructions' serial kernels at batch 1 (latency_ref phase: fresh GC, batch 1).
#   bash scripts/pmc_ref_b1.sh OUT
set -e
OUT=${1:-gpurun_out/pmc_ref_b1}
ROOT=$(pwd)
RE='k_sign_chain|k_rescale_update_approx|k_sign_castsum|k_sign_approx'
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --batch 1 --streams 1 --verify 0 --phases latency_ref --latency-gcs 2"
timeout -s KILL 300 rocprofv3 --kernel-trace --kernel-include-regex "$RE" \
    --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    --output-format csv -d "$ROOT/$OUT/a" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/a.log" 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --kernel-include-regex "$RE" \
    --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT \
    --output-format csv -d "$ROOT/$OUT/b" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/b.log" 2>&1
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT" > "$OUT/summary.txt"
rm -rf "$OUT/a" "$OUT/b"
cat "$OUT/summary.txt"
