#!/bin/bash
# full validation: every GPU test, smoke(), headline bench (main + reference constructions + served phases),
# batch-1 latency, served inferences/s vs concurrent garblings, kernel trace of the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3fin}
ROOT=$(pwd)
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --batch 1 --phases main > $OUT/b1.json 2> $OUT/b1.err || { tail -20 $OUT/b1.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('b1', d['value'], d['ms_per_step'], d['verified_vs_plaintext'])" $OUT/b1.json
WORKERS="${WORKERS:-4}" bash scripts/r3_serve.sh $T || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/kt" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --phases main > "$ROOT/$OUT/kt.log" 2>&1 || { tail -5 "$ROOT/$OUT/kt.log"; exit 1; }
cd "$ROOT"
DB=$(find $OUT/kt -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" 40 > $OUT/kt_summary.txt 2>&1 || true
rm -rf "$OUT/kt"
head -30 $OUT/kt_summary.txt
