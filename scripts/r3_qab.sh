#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
DISP=copyBuffer bash scripts/r3_q.sh ${1:-r3qab} && bash scripts/r3_hab.sh ${1:-r3qab}_ab
