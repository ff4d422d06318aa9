# GPU garbler: byte-identity tests vs the host garbler, offline timing, headline bench
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/gg
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ -k "gpu_garbler or smoke" > gpurun_out/gg/tests.log 2>&1
DASH_GG_TRACE=1 timeout -k 10 300 python -u scripts/garble_bench.py --reps 3 > gpurun_out/gg/garble.json 2> gpurun_out/gg/garble.err
if [ "${1:-}" = "bench" ]; then
  timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 > gpurun_out/gg/bench.json 2> gpurun_out/gg/bench.err
fi
