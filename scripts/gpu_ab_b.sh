#!/bin/bash
# per-op A/B (main vs ab/<variants>) at batch 24 and batch 1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-abb}
mkdir -p gpurun_out/$T
for B in 24 1; do
for d in . ab/*/; do
  n=$(basename "$d"); [ "$d" = . ] && n=main
  timeout -k 10 240 python scripts/ab_online.py --root "$d" --batch $B --steps 10 --relu joint --detail > gpurun_out/$T/${n}_b$B.json 2> gpurun_out/$T/${n}_b$B.err || { tail -20 gpurun_out/$T/${n}_b$B.err; exit 1; }
  echo "== $n b$B"; head -1 gpurun_out/$T/${n}_b$B.json
done
done
