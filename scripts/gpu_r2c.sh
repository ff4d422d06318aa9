#!/bin/bash
# GPU tests, then per-op online times: main (tap-unrolled conv on/off) and every ab/<variant>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r2c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
bash scripts/gpu_conv_ab.sh ${T}_ab
