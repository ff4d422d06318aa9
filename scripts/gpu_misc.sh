set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r2aa}
timeout -k 10 300 python bench.py --batch 1 --streams 1 --steps 20 --warmup 3 > gpurun_out/${T}_b1.json 2> gpurun_out/${T}_b1.err || { tail -5 gpurun_out/${T}_b1.err; exit 1; }
echo "batch1 $(cat gpurun_out/${T}_b1.json)"
DASH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --batch 8 --steps 3 --warmup 1 > gpurun_out/${T}_dp2.json 2> gpurun_out/${T}_dp2.err || { tail -20 gpurun_out/${T}_dp2.err; exit 1; }
echo "dp2 $(cat gpurun_out/${T}_dp2.json)"
