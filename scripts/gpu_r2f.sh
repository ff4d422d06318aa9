#!/bin/bash
# per-op A/B at batch 24 (main vs ab/<variants>), then smoke and the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r2f}
mkdir -p gpurun_out/$T
for d in . ab/*/; do
  n=$(basename "$d"); [ "$d" = . ] && n=main
  timeout -k 10 240 python scripts/ab_online.py --root "$d" --batch 24 --relu joint --detail > gpurun_out/$T/$n.json 2> gpurun_out/$T/$n.err || { tail -20 gpurun_out/$T/$n.err; exit 1; }
  echo "== $n"; head -1 gpurun_out/$T/$n.json
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
