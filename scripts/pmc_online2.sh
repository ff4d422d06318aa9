#!/bin/bash
# Online-evaluation PMC passes at the headline config (B GCs, 1 step + 1 warmup; kernels serialize under --pmc)
# usage: scripts/pmc_online2.sh OUTDIR [B] [bench dir]
set -e
OUT=${1:-gpurun_out/pmco2}
B=${2:-36}
D=${3:-.}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --batch $B --verify 0"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$ROOT/$OUT/f" -o run -- python3 "$ROOT/$D/bench.py" $ARGS > "$ROOT/$OUT/f.log" 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD --output-format csv -d "$ROOT/$OUT/w" -o run -- python3 "$ROOT/$D/bench.py" $ARGS > "$ROOT/$OUT/w.log" 2>&1
cd "$ROOT"
python3 -m dash_amd.utils.pmcsum $(find "$OUT/f" "$OUT/w" -name "*counter_collection.csv") > "$OUT/pmc.txt" 2>&1
cat "$OUT/pmc.txt"
