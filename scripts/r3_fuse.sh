#!/bin/bash
# staged fused joint rescale + ReLU kernel: parity tests, per-op times (fused vs two-kernel), headline main phase
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r3fuse}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_models.py -m gpu -x -q -k "joint or minionn or slot or full or streamed" --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for F in 1 0; do
  DASH_JOINT_FUSE=$F timeout -k 10 300 python scripts/ab_online.py --batch 24 --steps 5 --relu joint > gpurun_out/$T/ops_f$F.json 2> gpurun_out/$T/ops_f$F.err || { tail -20 gpurun_out/$T/ops_f$F.err; exit 1; }
  echo "fuse=$F $(head -1 gpurun_out/$T/ops_f$F.json)"
done
for F in 1 0; do
  DASH_JOINT_FUSE=$F timeout -k 10 400 python bench.py --steps 10 --warmup 3 --phases main > gpurun_out/$T/bench_f$F.json 2> gpurun_out/$T/bench_f$F.err || { tail -20 gpurun_out/$T/bench_f$F.err; exit 1; }
  echo "fuse=$F bench $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['config']['gcs_per_gpu'], d['verified_vs_plaintext'])" gpurun_out/$T/bench_f$F.json)"
done
