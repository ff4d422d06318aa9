#!/bin/bash
# PMC passes over the default online kernels (joint rescale+ReLU chain, output hash, relu multiply, conv) (bench, B GCs, 1 stream)
set -e
OUT=${1:-gpurun_out/pmcc}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --batch 24 --streams 1 --verify 0"
timeout -s KILL 200 rocprofv3 --kernel-trace --kernel-include-regex "k_mrs_chain|k_rescale_mrs_out_hash|k_relu_mult|k_conv_img2" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d "$ROOT/$OUT/a" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/a.log" 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --kernel-include-regex "k_mrs_chain|k_rescale_mrs_out_hash|k_relu_mult|k_conv_img2" --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --output-format csv -d "$ROOT/$OUT/b" -o run -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/b.log" 2>&1
cd "$ROOT"
python3 - "$OUT" <<'PY'
import csv, glob, sys, re
from collections import defaultdict
out = sys.argv[1]
agg = defaultdict(lambda: defaultdict(float)); ms = defaultdict(float); nd = defaultdict(int)
for f in glob.glob(f"{out}/*/**/*counter_collection.csv", recursive=True):
    seen = set()
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (f, r["Dispatch_Id"])
        if key not in seen:
            seen.add(key); ms[(k, f)] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6; nd[(k, f)] += 1
for k, c in agg.items():
    print(k)
    for n, v in sorted(c.items()): print(f"   {n:28s} {v:18.0f}")
for (k, f), v in ms.items(): print(k, f.split('/')[-3], f"{v:.2f} ms", nd[(k, f)], "dispatches")
PY
rm -rf "$OUT/a" "$OUT/b"
