#!/bin/bash
# Conv PMC of the online step (corrected MFMA utilisation, int8 TOPS) and a batch-1 PMC of the reference chain.
set -o pipefail
export TMPDIR=/tmp
bash scripts/pmc_conv.sh gpurun_out/r06v_conv 24 || exit 1
bash scripts/pmc_ref_b1.sh gpurun_out/r06v_ref || exit 1
