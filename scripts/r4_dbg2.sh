#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4dbg2
mkdir -p $OUT
export DASH_GG_TRACE=1
timeout -k 5 150 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 60 --timeout-method thread -k "test_gpu_garbler_bit_identical and (relu or sign or rescale or model_b)" > $OUT/t.log 2>&1; rc=$?
grep -v "^\[gg\]" $OUT/t.log | tail -60
echo "last gg lines:"; grep "^\[gg\]" $OUT/t.log | tail -5
echo rc=$rc
