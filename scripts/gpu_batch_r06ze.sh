#!/bin/bash
# Final tree validation: GPU tests, smoke, per-model garbling, full bench, two-party.
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_round.sh r06zu
