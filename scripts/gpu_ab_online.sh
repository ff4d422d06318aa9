#!/bin/bash
# ab_online.py for the main tree and every built ab/<variant>, back to back (one stream, no decode).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${1:-gpurun_out/abo}
B=${2:-24}
mkdir -p "$OUT"
for d in . ab/*/; do
  n=$(basename "$d"); [ "$d" = . ] && n=main
  timeout -k 10 240 python scripts/ab_online.py --root "$d" --batch $B > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -20 "$OUT/$n.err"; exit 1; }
  cat "$OUT/$n.json"
done
