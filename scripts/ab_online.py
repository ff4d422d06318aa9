"""Online-evaluation timing of one package tree (main or an ab/<variant> build), no decode.

    python scripts/ab_online.py --root ab/fake_dec --batch 24 --steps 5

Garbles B MiniONN GCs on the GPU, loads them into one evaluator (one stream),
then times `run` (upload of the encoded inputs + every layer) and prints one
JSON line with ms per step and the per-op-kind GPU times of a profiled run.
Outputs are never decoded, so an ab/ tree with a patched (wrong-result) kernel can still be timed;
such patches live only in the untracked ab/ copies, never in the production sources.
"""
import argparse
import json
import re
import os
import sys
import time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default=".")
    ap.add_argument("--batch", type=int, default=24)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--relu", default="approx")
    ap.add_argument("--detail", action="store_true", help="also print every op's time")
    args = ap.parse_args()
    sys.path.insert(0, os.path.abspath(args.root))
    import torch
    from dash_amd.garbling import GarbledCircuit
    from dash_amd.models import BENCH_CONFIGS, build_circuit, quantized_inputs
    from dash_amd.ir.quant import QuantizationMethod
    from dash_amd.runtime import HipEvaluator
    import dash_amd
    assert os.path.abspath(dash_amd.__file__).startswith(os.path.abspath(args.root)), dash_amd.__file__

    name = "MODEL_F_MINIONN_POOL_REPL"
    cfg = BENCH_CONFIGS[f"{name}/DASH"]
    qm = QuantizationMethod(cfg["q_method"])
    circuit = build_circuit(name, qm, cfg["q_parameter"], seed=0)
    B = args.batch
    xs = quantized_inputs(name, B, qm, cfg["q_parameter"], seed=3)
    gcs = [GarbledCircuit(circuit, cfg["crt"], cfg["mrs"], seed=bytes([b] * 16), device=0, rescale="mrs",
                          relu=args.relu) for b in range(B)]
    ev = HipEvaluator(template=gcs[0].model, batch=B, device=0)
    for b, gc in enumerate(gcs):
        ev.load(b, gc.model)
        ev.encode_compressed_into(b, gc, xs[b])
    st = torch.cuda.current_stream()
    for _ in range(2):
        ev.upload_inputs_compressed(st)
        ev.run(st)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        ev.upload_inputs_compressed(st)
        ev.run(st)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / args.steps
    ev.set_profile(True)
    ev.upload_inputs_compressed(st)
    ev.run(st)
    torch.cuda.synchronize()
    kinds = {}
    for op, t_ms in ev.op_times():
        k = op.rsplit(".", 1)[-1] if "." in op else re.sub(r"[0-9_#:]+", "", op)
        kinds[k] = round(kinds.get(k, 0.0) + t_ms, 3)
    print(json.dumps({"root": args.root, "batch": B, "ms_per_step": round(ms, 3), "ops": kinds}))
    if args.detail:
        print(json.dumps([(op, round(t_ms, 4)) for op, t_ms in ev.op_times()]))


if __name__ == "__main__":
    main()
