#!/bin/bash
# round-3 baseline: GPU tests, smoke, headline bench, GPU-garbler kernel trace (1 GC x 3)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3a}
ROOT=$(pwd)
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/$T/ggkt" -o run -- python3 -u "$ROOT/scripts/garble_bench.py" --reps 3 --gpu-only > "$ROOT/gpurun_out/$T/gg.txt" 2>&1 || { tail -20 "$ROOT/gpurun_out/$T/gg.txt"; exit 1; }
cd "$ROOT"
DB=$(find gpurun_out/$T/ggkt -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" 60 > gpurun_out/$T/gg_kt_summary.txt 2>&1 || true
rm -rf gpurun_out/$T/ggkt
cat gpurun_out/$T/gg.txt | tail -3
head -30 gpurun_out/$T/gg_kt_summary.txt
