#!/bin/bash
# conv epilogue (permlane-transposed 16-byte stores): parity tests, per-op times at 24 GCs, headline vs streams
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r3perm}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_models.py -m gpu -x -q -k "conv or minionn or model or joint or slot or full" --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
timeout -k 10 300 python scripts/ab_online.py --batch 24 --steps 5 --relu joint > gpurun_out/$T/ops.json 2> gpurun_out/$T/ops.err || { tail -20 gpurun_out/$T/ops.err; exit 1; }
head -1 gpurun_out/$T/ops.json
STREAMS="${STREAMS:-4 6 8}" bash scripts/r3_streams.sh $T
