#!/bin/bash
# headline bench vs the number of concurrent GC groups (streams)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r3str}
mkdir -p gpurun_out/$T
for S in ${STREAMS:-2 4 6 8}; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --phases main --streams $S > gpurun_out/$T/s$S.json 2> gpurun_out/$T/s$S.err || { tail -20 gpurun_out/$T/s$S.err; exit 1; }
  echo "streams $S $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['config']['gcs_per_gpu'], d['verified_vs_plaintext'])" gpurun_out/$T/s$S.json)"
done
