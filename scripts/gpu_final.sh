#!/bin/bash
# round-end validation: GPU tests, smoke, headline bench, batch-1 latency bench, per-op detail, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-fin}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
timeout -k 10 300 python bench.py --batch 1 --streams 1 --steps 20 --warmup 3 > gpurun_out/$T/bench_b1.json 2> gpurun_out/$T/bench_b1.err || { tail -20 gpurun_out/$T/bench_b1.err; exit 1; }
cat gpurun_out/$T/bench_b1.json
timeout -k 10 240 python scripts/ab_online.py --batch 24 --relu joint --detail > gpurun_out/$T/online_b24.json 2> gpurun_out/$T/online_b24.err || { tail -20 gpurun_out/$T/online_b24.err; exit 1; }
head -1 gpurun_out/$T/online_b24.json
bash scripts/prof_default.sh ${T}_prof > /dev/null || exit 1
head -12 gpurun_out/${T}_prof_kt_summary.txt
