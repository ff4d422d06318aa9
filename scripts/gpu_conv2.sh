set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r2o}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "conv or minionn_head" > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
bash scripts/prof_default.sh ${T} --streams 1 | grep -E "dev::|value" | cut -c1-150
