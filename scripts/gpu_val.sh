#!/bin/bash
# GPU validation: gpu tests, smoke, headline bench, one-stream online op times. Usage: gpu_val.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-val}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
timeout -k 10 240 python scripts/ab_online.py --batch 24 --relu joint > gpurun_out/${T}_online.json 2> gpurun_out/${T}_online.err || { tail -20 gpurun_out/${T}_online.err; exit 1; }
cat gpurun_out/${T}_online.json
timeout -k 10 240 python scripts/ab_online.py --batch 1 --steps 20 --relu joint > gpurun_out/${T}_online_b1.json 2> gpurun_out/${T}_online_b1.err || { tail -20 gpurun_out/${T}_online_b1.err; exit 1; }
cat gpurun_out/${T}_online_b1.json
