#!/bin/bash
# serving benchmark (fresh GC per inference, garbling pipelined, injected faults) and a 2-rank gloo rehearsal of bench.py on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-sdp}
mkdir -p gpurun_out/$T
timeout -k 10 400 python benchmarks/serving.py --slots 16 --groups 3 --faults 0.05 > gpurun_out/$T/serving.json 2> gpurun_out/$T/serving.err || { tail -20 gpurun_out/$T/serving.err; exit 1; }
tail -1 gpurun_out/$T/serving.json
DASH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 8 > gpurun_out/$T/dp2.json 2> gpurun_out/$T/dp2.err || { tail -20 gpurun_out/$T/dp2.err; exit 1; }
cat gpurun_out/$T/dp2.json
