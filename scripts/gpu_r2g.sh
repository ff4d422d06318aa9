#!/bin/bash
# GPU tests, per-op A/B (main vs ab/<variants>), headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r2g}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
bash scripts/gpu_ab_b.sh ${T}_ab || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
