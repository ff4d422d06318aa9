#!/bin/bash
# GPU garbler: phase trace (host waits) + PMC passes over the garbling kernels (sink mode, 4 GCs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3c}
ROOT=$(pwd)
OUT=gpurun_out/$T
mkdir -p $OUT
DASH_GG_TRACE=1 timeout -k 10 200 python -u scripts/garble_bench.py --sink 6 > $OUT/trace.json 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 1; }
tail -30 $OUT/trace.err
cd /tmp
RX="k_hash|k_emit|k_draw|k_bank"
N=0
run() {
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$RX" --pmc "$@" --output-format csv -d "$ROOT/$OUT/p$N" -o run -- python3 "$ROOT/scripts/garble_bench.py" --sink 3 > "$ROOT/$OUT/p$N.log" 2>&1 || { tail -5 "$ROOT/$OUT/p$N.log"; exit 1; }
  N=$((N+1))
}
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
run SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS
run TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum FETCH_SIZE
run WRITE_SIZE TCP_TCC_WRITE_REQ_sum
cd "$ROOT"
python3 -m dash_amd.utils.pmcsum $(find "$OUT" -name "*counter_collection.csv") > $OUT/pmc_summary.txt
cat $OUT/pmc_summary.txt
rm -rf "$OUT"/p?
