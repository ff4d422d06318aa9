#!/bin/bash
# conv parity tests, then the one-stream 24-GC step at several conv LDS budgets (DASH_CONV_LDS_KB)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-clds}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "conv or minionn or garbler" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for KB in ${KBS:-40}; do
  DASH_CONV_LDS_KB=$KB timeout -k 10 200 python scripts/ab_online.py --batch 24 --steps 10 > gpurun_out/${T}_$KB.json 2> gpurun_out/${T}_$KB.err || { tail -20 gpurun_out/${T}_$KB.err; exit 1; }
  echo "$KB $(cat gpurun_out/${T}_$KB.json)"
done
