set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r2l}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "conv or minionn or garbler" > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for V in 2 1; do
  DASH_CONV_IMG_VER=$V timeout -k 10 500 python bench.py --steps 10 --warmup 3 > gpurun_out/${T}_bench_v$V.json 2> gpurun_out/${T}_bench_v$V.err || { tail -20 gpurun_out/${T}_bench_v$V.err; exit 1; }
  echo "v$V $(python -c "import json;d=json.load(open('gpurun_out/${T}_bench_v$V.json'));print(d['value'], d['ms_per_step'], d['config']['gcs_per_gpu'])")"
done
