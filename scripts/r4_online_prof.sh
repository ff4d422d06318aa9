#!/bin/bash
# mixed-radix chain tests, online per-op profile at batch 1 and 24 (flagship constructions) with the latency
# staged chain on / off, kernel trace of the batch-1 run, bench latency phase
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=gpurun_out/r4op
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
ab() {  # name, env..., then ab_online args via AB_ARGS
  local name=$1; shift
  env "$@" timeout -k 10 300 python scripts/ab_online.py $AB_ARGS --steps 20 --relu joint --detail > $OUT/ops_$name.json 2> $OUT/ops_$name.err || { tail -5 $OUT/ops_$name.err; return 1; }
  echo "$name"; head -c 300 $OUT/ops_$name.json; echo
}
AB_ARGS="--batch 1" ab w1_b1 DASH_MRS_WAVE=1 && AB_ARGS="--batch 1" ab w1_b1_nofuse DASH_JOINT_FUSE=0 && \
AB_ARGS="--batch 1" ab w0_b1 DASH_MRS_WAVE=0 && AB_ARGS="--batch 24" ab w1_b24 DASH_MRS_WAVE=1 && \
AB_ARGS="--batch 24" ab w0_b24 DASH_MRS_WAVE=0 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/kt1" -o run -- python3 "$ROOT/scripts/ab_online.py" --root "$ROOT" --batch 1 --steps 50 --relu joint > "$ROOT/$OUT/kt1.log" 2>&1 || { tail -5 "$ROOT/$OUT/kt1.log"; exit 1; }
cd "$ROOT"
DB=$(find $OUT/kt1 -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" 30 > $OUT/kt1_summary.txt 2>&1 || true
rm -rf $OUT/kt1
head -16 $OUT/kt1_summary.txt
timeout -k 10 400 python bench.py --phases latency --steps 5 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
