#!/bin/bash
# ab_online.py --detail for the main tree and every built ab/<variant> (one stream, no decode): per-op times.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${1:-gpurun_out/abd}
B=${2:-24}
mkdir -p "$OUT"
for d in . ab/*/; do
  n=$(basename "$d"); [ "$d" = . ] && n=main
  timeout -k 10 240 python scripts/ab_online.py --root "$d" --batch $B --relu joint --detail > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -20 "$OUT/$n.err"; exit 1; }
  echo "== $n"; cat "$OUT/$n.json"
done
