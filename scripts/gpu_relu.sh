set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r2j}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "mrs" > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for R in mrs approx; do
  timeout -k 10 500 python bench.py --steps 10 --warmup 3 --relu $R > gpurun_out/${T}_bench_$R.json 2> gpurun_out/${T}_bench_$R.err || { tail -20 gpurun_out/${T}_bench_$R.err; exit 1; }
  echo "$R $(cat gpurun_out/${T}_bench_$R.json)"
done
