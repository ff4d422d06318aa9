#!/bin/bash
# garbler kernel A/B: hash kernel (entry | jobs) x AES copies (16 | 32), kernel trace of 4 sink GCs each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3hab}
ROOT=$(pwd)
mkdir -p gpurun_out/$T
for V in "entry 16" "entry 32" "jobs 16" "jobs 32"; do
  set -- $V
  cd /tmp
  DASH_GG_HASH=$1 DASH_GG_AES_COPIES=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/$T/kt_$1_$2" -o run -- python3 -u "$ROOT/scripts/garble_bench.py" --sink 4 > "$ROOT/gpurun_out/$T/gg_$1_$2.txt" 2>&1 || { tail -20 "$ROOT/gpurun_out/$T/gg_$1_$2.txt"; exit 1; }
  cd "$ROOT"
  DB=$(find gpurun_out/$T/kt_$1_$2 -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" 60 > gpurun_out/$T/kt_$1_$2.txt 2>&1 || true
  rm -rf gpurun_out/$T/kt_$1_$2
  echo "=== hash=$1 copies=$2"; head -8 gpurun_out/$T/kt_$1_$2.txt; grep TOTAL gpurun_out/$T/kt_$1_$2.txt
done
