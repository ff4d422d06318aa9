#!/bin/bash
# garbler: parity tests, sink timing of the hash / bank kernel variants, kernel trace of the default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3q2}
ROOT=$(pwd)
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_wire_compat.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -40 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
for V in ${VARIANTS:-"default default"}; do
  set -- $V
  timeout -k 10 300 env DASH_GG_HASH=$1 DASH_GG_BANK=$2 python -u scripts/garble_bench.py --sink 12 > gpurun_out/$T/gg_sink_$1_$2.json 2> gpurun_out/$T/gg_sink_$1_$2.err || { tail -20 gpurun_out/$T/gg_sink_$1_$2.err; exit 1; }
  echo "hash=$1 bank=$2 $(cut -c1-120 gpurun_out/$T/gg_sink_$1_$2.json)"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/$T/ggkt" -o run -- python3 -u "$ROOT/scripts/garble_bench.py" --sink 4 > "$ROOT/gpurun_out/$T/gg.txt" 2>&1 || { tail -20 "$ROOT/gpurun_out/$T/gg.txt"; exit 1; }
cd "$ROOT"
DB=$(find gpurun_out/$T/ggkt -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" 60 > gpurun_out/$T/gg_kt_summary.txt 2>&1 || true
rm -rf gpurun_out/$T/ggkt
head -24 gpurun_out/$T/gg_kt_summary.txt
if [ -n "$SERVE" ]; then
  timeout -k 10 300 python benchmarks/serving.py --slots 16 --groups 3 --requests 12 --faults 0.05 > gpurun_out/$T/serve.json 2> gpurun_out/$T/serve.err || { tail -20 gpurun_out/$T/serve.err; exit 1; }
  cat gpurun_out/$T/serve.json
fi
