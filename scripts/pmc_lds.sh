#!/bin/bash
# PMC passes over a one-group bench (B GCs, 1 stream): SQ issue/wait mix, LDS and memory counters.
set -e
OUT=${1:-gpurun_out/pmc2}
B=${2:-6}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$ROOT/$OUT/avail.txt" 2>&1 || true
run() {
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$ROOT/$OUT/$1" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --batch "$B" --streams 1 --verify 0 > "$ROOT/$OUT/$1.log" 2>&1
}
run SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD
run SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES
run FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE
