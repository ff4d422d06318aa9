#!/bin/bash
# quick garbler check: GPU garbler parity tests + kernel trace of 4 sink-mode GCs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3q}
ROOT=$(pwd)
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_wire_compat.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -40 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
timeout -k 10 300 python -u scripts/garble_bench.py --sink 12 > gpurun_out/$T/gg_sink.json 2> gpurun_out/$T/gg_sink.err || { tail -20 gpurun_out/$T/gg_sink.err; exit 1; }
cat gpurun_out/$T/gg_sink.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/$T/ggkt" -o run -- python3 -u "$ROOT/scripts/garble_bench.py" --sink 4 > "$ROOT/gpurun_out/$T/gg.txt" 2>&1 || { tail -20 "$ROOT/gpurun_out/$T/gg.txt"; exit 1; }
cd "$ROOT"
DB=$(find gpurun_out/$T/ggkt -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" 60 --dispatches "${DISP:-k_emit}" 40 > gpurun_out/$T/gg_kt_summary.txt 2>&1 || true
rm -rf gpurun_out/$T/ggkt
head -60 gpurun_out/$T/gg_kt_summary.txt
if [ -n "$AB16" ]; then
  cd /tmp
  DASH_GG_AES_COPIES=16 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/$T/ggkt16" -o run -- python3 -u "$ROOT/scripts/garble_bench.py" --sink 4 > "$ROOT/gpurun_out/$T/gg16.txt" 2>&1 || { tail -20 "$ROOT/gpurun_out/$T/gg16.txt"; exit 1; }
  cd "$ROOT"
  DB=$(find gpurun_out/$T/ggkt16 -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" 60 > gpurun_out/$T/gg_kt16_summary.txt 2>&1 || true
  rm -rf gpurun_out/$T/ggkt16
  echo "--- 16 copies"; head -8 gpurun_out/$T/gg_kt16_summary.txt
fi
