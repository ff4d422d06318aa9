#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench path on one GPU (gloo: RCCL refuses two ranks on one device)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r3dp2}
mkdir -p gpurun_out/$T
DASH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --batch 32 --phases main > gpurun_out/$T/dp2.json 2> gpurun_out/$T/dp2.err || { tail -20 gpurun_out/$T/dp2.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith(chr(123))][-1]); print(d['value'], d['n_gpus'], d['world_size'], d['dist_backend'], d['config']['global_batch'], d['config']['parallelism'], [(r['rank'], r['inf_per_s']) for r in d['ranks']], d['verified_vs_plaintext'])" gpurun_out/$T/dp2.json
