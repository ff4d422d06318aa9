#!/bin/bash
# joint rescale + ReLU: GPU parity tests, then the headline bench with --relu joint vs approx
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-joint}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "joint" > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --relu joint > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
timeout -k 10 240 python scripts/ab_online.py --batch 24 --relu joint > gpurun_out/${T}_online.json 2> gpurun_out/${T}_online.err || { tail -20 gpurun_out/${T}_online.err; exit 1; }
cat gpurun_out/${T}_online.json
timeout -k 10 240 python scripts/ab_online.py --batch 1 --steps 20 --relu joint > gpurun_out/${T}_online_b1.json 2> gpurun_out/${T}_online_b1.err || { tail -20 gpurun_out/${T}_online_b1.err; exit 1; }
cat gpurun_out/${T}_online_b1.json
