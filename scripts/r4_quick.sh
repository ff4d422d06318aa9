#!/bin/bash
# quick GPU check: parity / model tests, then per-op online profiles at the given batches
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/quick
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_models.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
for b in ${BATCHES:-1 24}; do
  timeout -k 10 300 python scripts/ab_online.py --batch $b --steps 20 --relu joint --detail > $OUT/ops_b$b.json 2> $OUT/ops_b$b.err || { tail -5 $OUT/ops_b$b.err; exit 1; }
  echo "b$b $(head -c 200 $OUT/ops_b$b.json)"
done
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py --phases $BENCH --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
  head -c 600 $OUT/bench.json; echo
fi
