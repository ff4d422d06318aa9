#!/bin/bash
# round 4: GPU garbler for every layer kind: byte-identity tests, whole models, per-model garble times
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r4gg}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_models.py -x -v --timeout 300 --timeout-method thread -k "${TESTS:-all_kinds or bit_identical or full_model}" > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for m in "VGG16 DASH" "RESNET18 DASH" "MODEL_F_MINIONN_POOL_REPL REDASH_OPT" "MODEL_F_MINIONN_POOL_REPL REDASH_CPM" "LENET5 DASH"; do
  set -- $m
  timeout -k 10 300 python bench.py --model $1 --config $2 --steps 3 --warmup 1 --phases main --batch ${BATCH:-16} --streams 4 > $OUT/bench_$1_$2.json 2> $OUT/bench_$1_$2.err || { tail -20 $OUT/bench_$1_$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['offline'], d['verified_vs_plaintext'], d['config']['rescale_construction'], d['config']['relu_construction'])" $OUT/bench_$1_$2.json
done
