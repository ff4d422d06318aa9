set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/gg
DASH_GG_TRACE=1 timeout -k 10 300 python -u scripts/garble_bench.py --reps 2 --gpu-only > gpurun_out/gg/trace.json 2> gpurun_out/gg/trace.err
