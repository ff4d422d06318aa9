"""Two-party deployment: garbler (client, holds the model secrets and the
inputs) and evaluator (server, holds the GPU) in separate processes.

Replaces the reference's only cross-boundary path, the SGX enclave <-> host
ocall split (sgx/Enclave/Enclave.edl:37-135, sgx/App/App.cpp), with a framed
TCP channel carrying exactly the protocol messages: the serialized
GarbledModel (offline) and one online round per inference (compressed input
labels -> compressed output labels), see SURVEY.md §2.3 M2-M6.
"""
from .channel import Channel, connect, listen  # noqa: F401
from .protocol import EvaluatorServer, GarblerClient  # noqa: F401
