"""dash_amd — MI355X-native arithmetic garbled circuits for private CNN inference.

A from-scratch rebuild of the capabilities of UzL-ITS/dash (DASH / ReDash):
CRT-residue label tensors, fixed-key-AES projection gates, approximate sign /
ReLU / rescale / base-extension gadgets, garbled dense and conv layers, a
host garbler emitting a serializable GarbledModel, a bit-exact host evaluator,
and a HIP/CDNA4 evaluator for gfx950 with RCCL batch data parallelism.
"""
from .ir.bases import first_primes, get_mrs_base  # noqa: F401
from .ir.circuit import Circuit  # noqa: F401
from .ir.layers import (Add, BaseExtension, Conv2d, Dense, Flatten, Max, MaxPool2d, MixedModMultLayer,  # noqa: F401
                        MultLayer, Projection, Relu, Rescale, Sign, SumPool2d)
from .ir.quant import QuantizationMethod  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    if name == "GarbledCircuit":
        from .garbling.gc import GarbledCircuit

        return GarbledCircuit
    if name == "IntegrityError":
        from .native import native

        return native().IntegrityError
    raise AttributeError(name)
