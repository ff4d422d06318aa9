#!/bin/bash
# headline phase at several GC-group counts (streams)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/streams
mkdir -p $OUT
for s in 8 12 6 16; do
  timeout -k 10 300 python bench.py --phases main --streams $s --steps 10 --warmup 3 > $OUT/s$s.json 2> $OUT/s$s.err || { tail -5 $OUT/s$s.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/s$s.json').readline()); print($s, d['value'], d['ms_per_step'])"
done
