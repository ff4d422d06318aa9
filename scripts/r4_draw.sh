#!/bin/bash
# GPU garbler after the chunk-major PRG draw: byte-identity tests, sink garble time, kernel trace, served phase
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=gpurun_out/draw
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
timeout -k 10 180 python scripts/garble_bench.py --sink 24 > $OUT/sink.json 2> $OUT/sink.err || { tail -20 $OUT/sink.err; exit 1; }
head -c 200 $OUT/sink.json; echo
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/kt" -o run -- python3 "$ROOT/scripts/garble_bench.py" --reps 4 --gpu-only > "$ROOT/$OUT/kt.log" 2>&1 || { tail -5 "$ROOT/$OUT/kt.log"; exit 1; }
cd "$ROOT"
DB=$(find $OUT/kt -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" 30 > $OUT/kt_summary.txt 2>&1 || true
rm -rf $OUT/kt
head -12 $OUT/kt_summary.txt
timeout -k 10 300 python bench.py --phases served --steps 5 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').readline()); print('served', d.get('served_inf_per_s'))"
