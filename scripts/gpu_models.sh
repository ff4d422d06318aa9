#!/bin/bash
# other models / schemes through the headline bench (default constructions, verified against the plaintext model)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-mod}
mkdir -p gpurun_out/$T
run() {
  n=$1; shift
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 "$@" > gpurun_out/$T/$n.json 2> gpurun_out/$T/$n.err || { tail -20 gpurun_out/$T/$n.err; exit 1; }
  echo "== $n"; python3 -c "import json,sys; d=json.load(open('gpurun_out/$T/$n.json')); print(d['value'], d['ms_per_inference'], d['config']['gcs_per_gpu'], d['verified_vs_plaintext'])"
}
run gnnp --model MODEL_F_GNNP_POOL_REPL
run redash_opt --config REDASH_OPT
run redash_cpm --config REDASH_CPM
run lenet5 --model LENET5
run vgg16 --model VGG16
run resnet18 --model RESNET18
