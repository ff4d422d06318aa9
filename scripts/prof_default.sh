# kernel trace + stats of the default headline bench (offline GPU garbling + online steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r2h}
shift || true
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/${T}_kt" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --verify 0 "$@" > "$ROOT/gpurun_out/${T}_kt_bench.json" 2> "$ROOT/gpurun_out/${T}_kt_bench.err" || { tail -5 "$ROOT/gpurun_out/${T}_kt_bench.err"; exit 1; }
cd "$ROOT"
DB=$(find gpurun_out/${T}_kt -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" > gpurun_out/${T}_kt_summary.txt 2>&1 || true
rm -rf gpurun_out/${T}_kt
cat gpurun_out/${T}_kt_summary.txt
cat gpurun_out/${T}_kt_bench.json
