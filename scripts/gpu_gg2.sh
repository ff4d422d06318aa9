set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r2v}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "garbler" > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
ROOT=$(pwd)
cd /tmp
cat > /tmp/gb.py <<'PY'
import time, sys
sys.path.insert(0, sys.argv[1])
from dash_amd.garbling import GarbledCircuit
from dash_amd.ir.quant import QuantizationMethod as Q
from dash_amd.models import build_circuit
c = build_circuit("MODEL_F_MINIONN_POOL_REPL", Q.ScaleQuant, 5, seed=0)
ts = []
for i in range(6):
    t = time.perf_counter(); g = GarbledCircuit(c, 7, 100.0, seed=bytes([i]) * 16, device=0, rescale="mrs"); ts.append(time.perf_counter() - t)
    g.model = None
print("garble s/GC", [round(x, 4) for x in ts])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/${T}_gg" -o run -- python3 /tmp/gb.py "$ROOT" > "$ROOT/gpurun_out/${T}_gb.log" 2>&1 || { tail "$ROOT/gpurun_out/${T}_gb.log"; exit 1; }
cd "$ROOT"
grep garble gpurun_out/${T}_gb.log
DB=$(find gpurun_out/${T}_gg -name "*.db" | head -n 1); python3 -m dash_amd.utils.profsum "$DB" > gpurun_out/${T}_gg_summary.txt 2>&1 || true
rm -rf gpurun_out/${T}_gg
head -20 gpurun_out/${T}_gg_summary.txt
