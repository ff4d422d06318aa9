#!/bin/bash
# Per-op online times (one stream) at batch 24 and 1, plus the batch-1 end-to-end latency bench. Usage: gpu_detail.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-det}
timeout -k 10 240 python scripts/ab_online.py --batch 24 --relu joint --detail > gpurun_out/${T}_online_b24.json 2> gpurun_out/${T}_online_b24.err || { tail -20 gpurun_out/${T}_online_b24.err; exit 1; }
timeout -k 10 240 python scripts/ab_online.py --batch 1 --steps 20 --relu joint --detail > gpurun_out/${T}_online_b1.json 2> gpurun_out/${T}_online_b1.err || { tail -20 gpurun_out/${T}_online_b1.err; exit 1; }
timeout -k 10 300 python bench.py --batch 1 --streams 1 --steps 20 --warmup 3 > gpurun_out/${T}_bench_b1.json 2> gpurun_out/${T}_bench_b1.err || { tail -20 gpurun_out/${T}_bench_b1.err; exit 1; }
cat gpurun_out/${T}_online_b24.json gpurun_out/${T}_online_b1.json gpurun_out/${T}_bench_b1.json
