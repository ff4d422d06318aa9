#!/bin/bash
# round-4 validation: every GPU test, smoke(), the default bench (all phases incl. thread sweep, batch-1
# latency, steady-state served), the --gpus 2 refusal on a 1-GPU box, and a PMC roofline of the GPU garbler
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r4chk}
ROOT=$(pwd)
OUT=gpurun_out/$T
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
fi
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
# a 2-GPU request on a 1-GPU box must fail loudly (exit 2), not measure one GPU
timeout -k 10 120 python bench.py --gpus 2 --steps 1 > $OUT/gpus2.out 2> $OUT/gpus2.err; rc=$?
echo "gpus2 rc=$rc"; tail -2 $OUT/gpus2.err
[ $rc -eq 2 ] || exit 1
if [ "${PMC:-1}" = 1 ]; then
  bash scripts/pmc_garble3.sh $OUT/pmcg > $OUT/pmc_garble.txt 2>&1 || { tail -20 $OUT/pmc_garble.txt; exit 1; }
  cat $OUT/pmc_garble.txt
fi
