#!/usr/bin/env python
"""Headline benchmark: online garbled inferences/sec for the MiniONN-style
CIFAR-10 CNN (MODEL_F_MINIONN_POOL_REPL, DASH config: ScaleQuant l=5, k=7 CRT
base {2..17}, ReLU accuracy 100 %).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Prints one JSON line (rank 0). The driver, timed region, phases (headline,
reference constructions, fresh-GC serving) and the multi-rank evidence live in
dash_amd/benchcore.py, which the multi-rank CPU tests run as well.
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from dash_amd.benchcore import main  # noqa: E402

if __name__ == "__main__":
    main()
