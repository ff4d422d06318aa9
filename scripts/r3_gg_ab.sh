#!/bin/bash
# garbler parity + whole-model/streamed-table GPU tests, sink timing of garbler variants (env knobs), kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3ggab}
ROOT=$(pwd)
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_wire_compat.py tests/test_gpu_models.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -40 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
for V in "default default" "jobs default" "default row"; do
  set -- $V
  timeout -k 10 300 env DASH_GG_HASH=$1 DASH_GG_BANK=$2 python -u scripts/garble_bench.py --sink 12 > gpurun_out/$T/gg_sink_$1_$2.json 2> gpurun_out/$T/gg_sink_$1_$2.err || { tail -20 gpurun_out/$T/gg_sink_$1_$2.err; exit 1; }
  echo "hash=$1 bank=$2 $(cat gpurun_out/$T/gg_sink_$1_$2.json)"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/$T/ggkt" -o run -- python3 -u "$ROOT/scripts/garble_bench.py" --sink 4 > "$ROOT/gpurun_out/$T/gg.txt" 2>&1 || { tail -20 "$ROOT/gpurun_out/$T/gg.txt"; exit 1; }
cd "$ROOT"
DB=$(find gpurun_out/$T/ggkt -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" 60 --dispatches copyBuffer 40 > gpurun_out/$T/gg_kt_summary.txt 2>&1 || true
rm -rf gpurun_out/$T/ggkt
head -64 gpurun_out/$T/gg_kt_summary.txt
# online: staged chain vs per-lane chain, 24-GC step and the default batch (verified against plaintext)
for S in 1 0; do
  timeout -k 10 300 env DASH_MRS_STAGE=$S python bench.py --steps 10 --warmup 2 --batch 24 --phases main > gpurun_out/$T/b24_stage$S.json 2> gpurun_out/$T/b24_stage$S.err || { tail -20 gpurun_out/$T/b24_stage$S.err; exit 1; }
  echo "stage=$S b24 $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['verified_vs_plaintext'])" gpurun_out/$T/b24_stage$S.json)"
done
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
