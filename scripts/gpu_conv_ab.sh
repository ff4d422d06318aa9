#!/bin/bash
# Per-op online times: main with/without the tap-unrolled conv, and every ab/<variant> without it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-cab}
mkdir -p gpurun_out/$T
for u in 1 0; do
  DASH_CONV_UNROLL=$u timeout -k 10 240 python scripts/ab_online.py --batch 24 --relu joint --detail > gpurun_out/$T/main_u$u.json 2> gpurun_out/$T/main_u$u.err || { tail -20 gpurun_out/$T/main_u$u.err; exit 1; }
  echo "== main unroll=$u"; cat gpurun_out/$T/main_u$u.json
done
for d in ab/*/; do
  n=$(basename "$d")
  DASH_CONV_UNROLL=0 timeout -k 10 240 python scripts/ab_online.py --root "$d" --batch 24 --relu joint --detail > gpurun_out/$T/$n.json 2> gpurun_out/$T/$n.err || { tail -20 gpurun_out/$T/$n.err; exit 1; }
  echo "== $n"; cat gpurun_out/$T/$n.json
done
