# GPU garbler check: byte-identical vs host garbler, per-GC time, kernel profile, headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r2c}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "garbler or conv or rescale_legacy or relu" > gpurun_out/${T}_gg_tests.log 2>&1 || { tail -40 gpurun_out/${T}_gg_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gg_tests.log
timeout -k 10 300 python -u scripts/garble_bench.py --reps 3 > gpurun_out/${T}_garble.json 2>&1 || { tail -20 gpurun_out/${T}_garble.json; exit 1; }
cat gpurun_out/${T}_garble.json
ROOT=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/${T}_ggkt" -o run -- python3 "$ROOT/scripts/garble_bench.py" --reps 3 --gpu-only > "$ROOT/gpurun_out/${T}_ggkt.log" 2>&1 || exit 1
cd "$ROOT"
DB=$(find gpurun_out/${T}_ggkt -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" > gpurun_out/${T}_ggkt_summary.txt 2>&1 || true
head -30 gpurun_out/${T}_ggkt_summary.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
