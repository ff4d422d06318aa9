#!/bin/bash
# PMC of the batch-1 online kernels (MiniONN, flagship constructions) -> summary on stdout
set -e
OUT=${1:-gpurun_out/pmcb1}
B=${2:-1}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
RX="k_mrs_chain|k_rescale|k_relu|k_conv"
run() {
  timeout -s KILL 150 rocprofv3 --kernel-trace --kernel-include-regex "$RX" --pmc "$@" --output-format csv -d "$ROOT/$OUT/p$N" -o run -- python3 "$ROOT/scripts/ab_online.py" --root "$ROOT" --batch $B --steps 10 --relu joint > "$ROOT/$OUT/p$N.log" 2>&1
  N=$((N+1))
}
N=0
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
run SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS
run SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_IFETCH SQ_INST_LEVEL_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_EXP
cd "$ROOT"
python3 -m dash_amd.utils.pmcsum $(find "$OUT" -name "*counter_collection.csv")
rm -rf "$OUT"/p?
