set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r2_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r2_gpu_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2_bench_fused.json 2> gpurun_out/r2_bench_fused.err || { tail -20 gpurun_out/r2_bench_fused.err; exit 1; }
cat gpurun_out/r2_bench_fused.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --sign reference --batch 28 > gpurun_out/r2_bench_ref.json 2> gpurun_out/r2_bench_ref.err || { tail -20 gpurun_out/r2_bench_ref.err; exit 1; }
cat gpurun_out/r2_bench_ref.json
