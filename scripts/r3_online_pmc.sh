#!/bin/bash
# Online roofline: kernel trace + PMC passes (time, wave states, instruction mix, HBM bytes) over the online
# kernels of a 24-GC MiniONN step (one stream), summarised per kernel by dash_amd.utils.pmcsum
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3on}
ROOT=$(pwd)
OUT=gpurun_out/$T
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --batch 24 --streams 1 --verify 0 --phases main"
RX="${RX:-k_mrs_chain|k_rescale_relu_out|k_rescale_mrs_out|k_relu_mult|k_conv_img2|k_sign_|k_dense|k_maxpool|k_unpack|k_label_hash}"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/kt" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/kt.log" 2>&1 || { tail -5 "$ROOT/$OUT/kt.log"; exit 1; }
N=0
run() {
  timeout -s KILL 200 rocprofv3 --kernel-trace --kernel-include-regex "$RX" --pmc "$@" --output-format csv -d "$ROOT/$OUT/p$N" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/p$N.log" 2>&1 || { tail -5 "$ROOT/$OUT/p$N.log"; exit 1; }
  N=$((N+1))
}
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
run SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS
run FETCH_SIZE
run WRITE_SIZE
cd "$ROOT"
DB=$(find $OUT/kt -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" 40 > $OUT/kt_summary.txt 2>&1 || true
python3 -m dash_amd.utils.pmcsum $(find "$OUT" -name "*counter_collection.csv") > $OUT/pmc_summary.txt
head -30 $OUT/kt_summary.txt
cat $OUT/pmc_summary.txt
rm -rf "$OUT"/p? "$OUT/kt"
