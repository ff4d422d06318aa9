#!/bin/bash
# GPU tests, sink-mode garbler trace (12 GCs into evaluator slots), headline bench (3 phases)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3b}
ROOT=$(pwd)
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -40 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
timeout -k 10 300 python -u scripts/garble_bench.py --sink 12 > gpurun_out/$T/gg_sink.json 2> gpurun_out/$T/gg_sink.err || { tail -20 gpurun_out/$T/gg_sink.err; exit 1; }
cat gpurun_out/$T/gg_sink.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/$T/ggkt" -o run -- python3 -u "$ROOT/scripts/garble_bench.py" --sink 4 > "$ROOT/gpurun_out/$T/gg.txt" 2>&1 || { tail -20 "$ROOT/gpurun_out/$T/gg.txt"; exit 1; }
cd "$ROOT"
DB=$(find gpurun_out/$T/ggkt -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" 60 --dispatches k_project 40 > gpurun_out/$T/gg_kt_summary.txt 2>&1 || true
rm -rf gpurun_out/$T/ggkt
head -24 gpurun_out/$T/gg_kt_summary.txt
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
timeout -k 10 300 python benchmarks/serving.py --slots 16 --groups 3 --requests 12 --faults 0.05 > gpurun_out/$T/serve.json 2> gpurun_out/$T/serve.err || { tail -20 gpurun_out/$T/serve.err; exit 1; }
cat gpurun_out/$T/serve.json
