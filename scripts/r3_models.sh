#!/bin/bash
# other models / schemes on the round-3 kernels (main phase, default constructions, verified against the
# plaintext model) + the MFMA-vs-VALU dense micro sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r3mod}
mkdir -p gpurun_out/$T
run() {
  n=$1; shift
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --phases main "$@" > gpurun_out/$T/$n.json 2> gpurun_out/$T/$n.err || { tail -20 gpurun_out/$T/$n.err; exit 1; }
  echo "== $n $(python3 -c "import json,sys; d=json.load(open('gpurun_out/$T/$n.json')); print(d['value'], d['ms_per_inference'], d['config']['gcs_per_gpu'], d['offline']['table_gb_per_gc'], d['verified_vs_plaintext'])")"
}
run model_a --model MODEL_A --config DASH
run gnnp --model MODEL_F_GNNP_POOL_REPL
run redash_opt --config REDASH_OPT
run redash_cpm --config REDASH_CPM
run lenet5 --model LENET5
run vgg16 --model VGG16
run resnet18 --model RESNET18
timeout -k 10 300 python benchmarks/micro.py --layers dense --targets gpu,gpu_valu --batch 16 --runs 3 --out gpurun_out/$T/micro > gpurun_out/$T/micro.log 2>&1 || { tail -20 gpurun_out/$T/micro.log; exit 1; }
tail -15 gpurun_out/$T/micro.log
