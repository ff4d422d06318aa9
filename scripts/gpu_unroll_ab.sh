#!/bin/bash
# GPU tests, then per-op online times with and without the tap-unrolled conv image (env A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-ur}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
for u in 1 0; do
  DASH_CONV_UNROLL=$u timeout -k 10 240 python scripts/ab_online.py --batch 24 --relu joint --detail > gpurun_out/${T}_u$u.json 2> gpurun_out/${T}_u$u.err || { tail -20 gpurun_out/${T}_u$u.err; exit 1; }
  echo "== unroll=$u"; cat gpurun_out/${T}_u$u.json
done
