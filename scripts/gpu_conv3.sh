set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r2t}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "conv or minionn_head" > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for KB in 64 40 32 24; do
  DASH_CONV_LDS_KB=$KB timeout -k 10 500 python bench.py --steps 2 --warmup 1 --streams 1 --profile --verify 0 > gpurun_out/${T}_p$KB.json 2> gpurun_out/${T}_p$KB.err || { tail -5 gpurun_out/${T}_p$KB.err; exit 1; }
  python - gpurun_out/${T}_p$KB.json $KB <<'PY'
import json,sys
d=json.load(open(sys.argv[1])); ops=d['op_ms']
conv=sum(v for n,v in ops if n.startswith('conv'))
print(sys.argv[2], "KB: inf/s", d['value'], "conv ms/step", round(conv,2), "total", round(sum(v for _,v in ops),2))
PY
done
