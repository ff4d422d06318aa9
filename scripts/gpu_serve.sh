set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r2w}
for CFG in "--slots 8 --groups 3" "--slots 16 --groups 3"; do
  timeout -k 10 400 python benchmarks/serving.py $CFG --requests 12 --faults 0.05 > gpurun_out/${T}_serve.json 2> gpurun_out/${T}_serve.err || { tail -20 gpurun_out/${T}_serve.err; exit 1; }
  echo "$CFG $(cat gpurun_out/${T}_serve.json)"
done
