#!/bin/bash
# PMC passes behind docs/ROOFLINE.md (run on the GPU box from the repo root):
#   flagship online kernels at 24 GCs (one stream) and 160 GCs (8 streams), and the reference-constructions
#   kernels at 24 GCs. Each pass is pmc_kernels.sh (kernel trace + counters, one bench step).
set -o pipefail
OUT=${1:-gpurun_out/roof}
mkdir -p "$OUT"
FLAG='k_mrs_chain|k_rescale_mrs_out_hash|k_relu_mult|k_conv_img2|k_rescale_relu_out'
REF='k_sign_chain|k_rescale_update_approx|k_sign_castsum|k_sign_approx|k_rescale_hash'
bash scripts/pmc_kernels.sh "$OUT/flag24" "$FLAG" 24 > "$OUT/flag24.log" 2>&1 || { tail -20 "$OUT/flag24.log"; exit 1; }
STREAMS=8 bash scripts/pmc_kernels.sh "$OUT/flag160" "$FLAG" 160 > "$OUT/flag160.log" 2>&1 || { tail -20 "$OUT/flag160.log"; exit 1; }
EXTRA="--constructions reference" bash scripts/pmc_kernels.sh "$OUT/ref24" "$REF" 24 > "$OUT/ref24.log" 2>&1 || { tail -20 "$OUT/ref24.log"; exit 1; }
echo done
