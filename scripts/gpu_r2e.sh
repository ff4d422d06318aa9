#!/bin/bash
# GPU tests, then per-op online times at batch 24: main, main with the fused joint ReLU forced on, ab/<variants>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r2e}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
for f in -1 1; do
  DASH_JOINT_FUSE=$f timeout -k 10 240 python scripts/ab_online.py --batch 24 --relu joint --detail > gpurun_out/$T/main_f$f.json 2> gpurun_out/$T/main_f$f.err || { tail -20 gpurun_out/$T/main_f$f.err; exit 1; }
  echo "== main fuse=$f"; head -1 gpurun_out/$T/main_f$f.json
done
for d in ab/*/; do
  n=$(basename "$d")
  timeout -k 10 240 python scripts/ab_online.py --root "$d" --batch 24 --relu joint --detail > gpurun_out/$T/$n.json 2> gpurun_out/$T/$n.err || { tail -20 gpurun_out/$T/$n.err; exit 1; }
  echo "== $n"; head -1 gpurun_out/$T/$n.json
done
timeout -k 10 240 python scripts/ab_online.py --batch 1 --steps 20 --relu joint --detail > gpurun_out/$T/main_b1.json 2> gpurun_out/$T/main_b1.err || { tail -20 gpurun_out/$T/main_b1.err; exit 1; }
echo "== main b1"; head -1 gpurun_out/$T/main_b1.json
