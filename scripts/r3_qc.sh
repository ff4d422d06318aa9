#!/bin/bash
# quick garbler check + PMC passes over the projection kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/r3_q.sh ${1:-r3qc} && bash scripts/r3_c.sh ${1:-r3qc}_pmc
