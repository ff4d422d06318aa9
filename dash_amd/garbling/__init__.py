"""Garbling API (GarbledCircuit) on top of the native garbler/evaluator."""
from .gc import GarbledCircuit, ReferenceEncodingWarning, garble  # noqa: F401
from .guard import RangeGuard, RangeGuardError  # noqa: F401
