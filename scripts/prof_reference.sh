set -o pipefail
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out/r06_ref
PHASES=reference EXTRA="--ref-batch 24 --ref-steps 3" timeout -k 10 400 bash scripts/prof_bench.sh gpurun_out/r06_ref/b24 8 || exit 1
PHASES=latency_ref AFTER=gg:: EXTRA="--latency-gcs 3" timeout -k 10 400 bash scripts/prof_bench.sh gpurun_out/r06_ref/lat 8 || exit 1
tail -3 gpurun_out/r06_ref/b24/summary.txt gpurun_out/r06_ref/lat/summary.txt
