#!/bin/bash
# PMC passes over the online conv kernels (24 GCs, one stream, scripts/ab_online.py) -> summary on stdout
set -e
OUT=${1:-gpurun_out/pmcc2}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
RX="k_conv_img2"
run() {
  timeout -s KILL 150 rocprofv3 --kernel-trace --kernel-include-regex "$RX" --pmc "$@" --output-format csv -d "$ROOT/$OUT/p$N" -o run -- python3 "$ROOT/scripts/ab_online.py" --root "$ROOT" --batch 24 --steps 1 > "$ROOT/$OUT/p$N.log" 2>&1
  N=$((N+1))
}
N=0
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES
run SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA
run FETCH_SIZE
run WRITE_SIZE
cd "$ROOT"
python3 -m dash_amd.utils.pmcsum $(find "$OUT" -name "*counter_collection.csv")
mkdir -p "$OUT/csv"; i=0; for f in $(find "$OUT" -name "*counter_collection.csv"); do cp "$f" "$OUT/csv/c$i.csv"; i=$((i+1)); done; rm -rf "$OUT"/p?
