#!/bin/bash
# garbler check: parity tests, sink timing, kernel trace (default) + sink timing and trace with DASH_GG_BANK=row (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3bank}
ROOT=$(pwd)
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_wire_compat.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -40 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
for V in default row; do
  timeout -k 10 300 env DASH_GG_BANK=$V python -u scripts/garble_bench.py --sink 12 > gpurun_out/$T/gg_sink_$V.json 2> gpurun_out/$T/gg_sink_$V.err || { tail -20 gpurun_out/$T/gg_sink_$V.err; exit 1; }
  echo "$V $(cat gpurun_out/$T/gg_sink_$V.json)"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/$T/ggkt" -o run -- python3 -u "$ROOT/scripts/garble_bench.py" --sink 4 > "$ROOT/gpurun_out/$T/gg.txt" 2>&1 || { tail -20 "$ROOT/gpurun_out/$T/gg.txt"; exit 1; }
cd "$ROOT"
DB=$(find gpurun_out/$T/ggkt -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" 60 > gpurun_out/$T/gg_kt_summary.txt 2>&1 || true
rm -rf gpurun_out/$T/ggkt
head -24 gpurun_out/$T/gg_kt_summary.txt
