#!/bin/bash
# HIP API trace of 2 sink-mode garblings: which runtime calls issue the blit (copyBuffer) kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=gpurun_out/${1:-r3ct}
mkdir -p $OUT
cd /tmp
timeout -k 10 240 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d "$ROOT/$OUT/t" -o run -- python3 "$ROOT/scripts/garble_bench.py" --sink 2 > "$ROOT/$OUT/t.log" 2>&1 || { tail -5 "$ROOT/$OUT/t.log"; exit 1; }
cd "$ROOT"
F=$(find $OUT/t -name "*hip_api_trace.csv" | head -n 1)
python3 - "$F" > $OUT/api_summary.txt <<'PY'
import csv, sys, collections
c = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    n = r.get("Function") or r.get("Operation") or ""
    if "emcpy" in n or "emset" in n or "Malloc" in n or "Free" in n:
        c[n] += 1
for k, v in c.most_common(30):
    print(f"{v:8d}  {k}")
PY
cat $OUT/api_summary.txt
rm -rf $OUT/t
