#!/bin/bash
# conv bound analysis: per-op online times (24 GCs, joint ReLU) of the main build and stand-in builds
# (main: 32 filters per wave; ab/conv_fw16: 16; ab/conv_noldsb: MFMA B operands from registers; conv_noload: band staging without global loads;
#  conv_nostore: epilogue without stores) -- stand-ins give wrong outputs, nothing is decoded
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r3cab}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "conv or minionn or model or joint or slot" --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for V in . ab/conv_fw16 ab/conv_noldsb ab/conv_noload ab/conv_nostore; do
  n=$(basename $V); [ "$V" = "." ] && n=main
  timeout -k 10 300 python scripts/ab_online.py --root $V --batch 24 --steps 5 --relu joint > gpurun_out/$T/$n.json 2> gpurun_out/$T/$n.err || { tail -20 gpurun_out/$T/$n.err; exit 1; }
  echo "$n $(head -1 gpurun_out/$T/$n.json)"
done
