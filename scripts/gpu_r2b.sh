set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2b_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r2b_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r2b_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2b_smoke.log 2>&1 || { tail -20 gpurun_out/r2b_smoke.log; exit 1; }
tail -2 gpurun_out/r2b_smoke.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r2b_bench.json 2> gpurun_out/r2b_bench.err || { tail -20 gpurun_out/r2b_bench.err; exit 1; }
cat gpurun_out/r2b_bench.json
ROOT=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r2b_kt" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --verify 0 > "$ROOT/gpurun_out/r2b_kt_bench.json" 2> "$ROOT/gpurun_out/r2b_kt_bench.err" || exit 1
cd "$ROOT"
DB=$(find gpurun_out/r2b_kt -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" > gpurun_out/r2b_kt_summary.txt 2>&1 || true
head -40 gpurun_out/r2b_kt_summary.txt
