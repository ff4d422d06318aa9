#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4dbg
mkdir -p $OUT
export DASH_GG_TRACE=1 DASH_GG_SYNC=1
for case in "dense 2" "dense_relu 2" "model_b 0" "model_b 2"; do
  set -- $case
  echo "== $1 keys=$2"
  DASH_GG_KEYS=$2 timeout -k 5 60 python -u scripts/r4_dbg.py $1 > $OUT/$1_$2.log 2>&1; rc=$?
  tail -25 $OUT/$1_$2.log; echo "rc=$rc"
  [ $rc -eq 0 ] || exit 1
done
