#!/bin/bash
# served inferences/s (fresh GC per inference, 5 % injected faults) vs the number of concurrent GPU garblings
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r3serve}
mkdir -p gpurun_out/$T
for W in ${WORKERS:-2 3 4}; do
  DASH_GG_CONTEXTS=$W timeout -k 10 300 python benchmarks/serving.py --slots 16 --groups 3 --requests 12 --faults 0.05 --garble-workers $W > gpurun_out/$T/serve_w$W.json 2> gpurun_out/$T/serve_w$W.err || { tail -20 gpurun_out/$T/serve_w$W.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('workers', d['garble_workers'], 'wall inf/s', d['inferences_per_s_wall'], 'garble s/GC', d['garble_s_per_gc'], 'ok', d['ok'])" gpurun_out/$T/serve_w$W.json
done
