#!/bin/bash
# GPU-garbler sink-mode timing (12 GCs) of the main tree and every ab/<variant> build, back to back
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-abg}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 200 python scripts/garble_bench.py --sink 12 > $OUT/main.json 2> $OUT/main.err || { tail -20 $OUT/main.err; exit 1; }
echo "main $(cat $OUT/main.json)"
for d in ab/*/; do
  n=$(basename "$d")
  DASH_PKG_ROOT=$d timeout -k 10 200 python scripts/garble_bench.py --sink 12 > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
  echo "$n $(cat $OUT/$n.json)"
done
timeout -k 10 200 python scripts/garble_bench.py --sink 12 > $OUT/main2.json 2> $OUT/main2.err || { tail -20 $OUT/main2.err; exit 1; }
echo "main2 $(cat $OUT/main2.json)"
