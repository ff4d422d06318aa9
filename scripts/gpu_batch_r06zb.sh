#!/bin/bash
# Final tree: GPU tests, smoke, full bench (new defaults: 4 pipelined groups, reference phase on 2 groups).
set -o pipefail
export TMPDIR=/tmp
SKIP_GARBLE=1 SKIP_TP=1 bash scripts/gpu_round.sh r06zb
