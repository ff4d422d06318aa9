# rocprofv3 kernel summary of the GPU garbler (one MiniONN GC, 2 reps + warmup), CSV stats
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ggprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ggprof -o run -- python3 -u scripts/garble_bench.py --reps 2 --gpu-only > gpurun_out/ggprof/out.txt 2>&1
