#!/bin/bash
# conv knobs at batch 24: staging items per round trip (ab/<variants>) and the LDS band budget (env)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-ck}
mkdir -p gpurun_out/$T
for d in . ab/*/; do
  n=$(basename "$d"); [ "$d" = . ] && n=main
  timeout -k 10 240 python scripts/ab_online.py --root "$d" --batch 24 --steps 10 --relu joint --detail > gpurun_out/$T/$n.json 2> gpurun_out/$T/$n.err || { tail -20 gpurun_out/$T/$n.err; exit 1; }
  echo "== $n"; head -1 gpurun_out/$T/$n.json
done
for kb in 24 32 56; do
  DASH_CONV_LDS_KB=$kb timeout -k 10 240 python scripts/ab_online.py --batch 24 --steps 10 --relu joint --detail > gpurun_out/$T/lds$kb.json 2> gpurun_out/$T/lds$kb.err || { tail -20 gpurun_out/$T/lds$kb.err; exit 1; }
  echo "== lds $kb"; head -1 gpurun_out/$T/lds$kb.json
done
