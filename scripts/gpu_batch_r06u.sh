#!/bin/bash
# Round-6 validation of the final tree: GPU tests, smoke, per-model garbling, full bench, two-party; then a kernel
# trace of the headline step.
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_round.sh r06u || exit 1
bash scripts/prof_bench.sh gpurun_out/r06u_prof 160 && head -30 gpurun_out/r06u_prof/summary.txt
