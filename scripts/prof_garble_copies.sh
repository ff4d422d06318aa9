#!/bin/bash
# Memory-copy and kernel trace of the GPU garbler (4 MiniONN GCs, gpu only): which copies run per GC and how big.
set -o pipefail
OUT=${1:-gpurun_out/gcopy}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$ROOT/$OUT/db" -o run -- \
    python3 "$ROOT/scripts/garble_bench.py" --gpu-only --reps 4 > "$ROOT/$OUT/run.log" 2>&1 || { tail -20 "$ROOT/$OUT/run.log"; exit 1; }
cd "$ROOT"
python3 - "$OUT" <<'PY'
import glob, sqlite3, sys, collections
db = glob.glob(sys.argv[1] + "/db/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
print("tables:", [t for t in tabs if "copy" in t.lower() or "memory" in t.lower()][:20])
for t in tabs:
    if "memory_copy" in t.lower() and not t.lower().startswith("rocpd_info"):
        cols = [r[1] for r in c.execute(f"pragma table_info('{t}')")]
        print(t, cols[:30])
        rows = c.execute(f"select * from '{t}' limit 5").fetchall()
        for r in rows: print(r)
        break
PY
