"""Garbling API (GarbledCircuit) on top of the native garbler/evaluator."""
from .gc import GarbledCircuit, ReferenceEncodingWarning, garble  # noqa: F401
