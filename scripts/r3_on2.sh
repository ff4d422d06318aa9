#!/bin/bash
# online per-op breakdown (24 GCs, joint ReLU) staged vs per-lane, PMC of the staged kernels, batch-1 latency
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3on2}
ROOT=$(pwd)
OUT=gpurun_out/$T
mkdir -p $OUT
for S in 1 0; do
  DASH_MRS_STAGE=$S timeout -k 10 300 python scripts/ab_online.py --batch 24 --steps 5 --relu joint --detail > $OUT/ops_stage$S.json 2> $OUT/ops_stage$S.err || { tail -20 $OUT/ops_stage$S.err; exit 1; }
  head -1 $OUT/ops_stage$S.json
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --batch 1 --phases main > $OUT/b1.json 2> $OUT/b1.err || { tail -20 $OUT/b1.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('b1', d['value'], d['ms_per_step'], d['verified_vs_plaintext'])" $OUT/b1.json
ARGS="--steps 2 --warmup 1 --batch 24 --streams 1 --verify 0 --phases main"
RX="${RX:-k_mrs_chain|k_rescale_mrs_out|k_relu_mult|k_conv_img2}"
cd /tmp
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
python3 -m dash_amd.utils.pmcsum $(find "$OUT" -name "*counter_collection.csv") > $OUT/pmc_summary.txt
cat $OUT/pmc_summary.txt
rm -rf "$OUT"/p?
