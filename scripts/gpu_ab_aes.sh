# A/B: AES LDS image copies (32 = main build, 16, 8) on the headline bench + garble time
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r2d}
for V in main aes16 aes8; do
  if [ $V = main ]; then D=.; else D=ab/$V; fi
  timeout -k 10 300 python $D/bench.py --steps 10 --warmup 3 > gpurun_out/${T}_bench_$V.json 2> gpurun_out/${T}_bench_$V.err || { tail -20 gpurun_out/${T}_bench_$V.err; exit 1; }
  echo "$V $(cat gpurun_out/${T}_bench_$V.json | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["offline"])')"
done
