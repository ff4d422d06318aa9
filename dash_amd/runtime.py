"""GPU evaluator front-end (HIP / gfx950).

`HipEvaluator` evaluates a *batch* of garbled models of the same circuit in
one pass: every kernel launch covers (GC x residue x element), tables of all
GCs sit in one HBM arena. Input/output labels use the same host format as the
CPU evaluator: per residue a tuple (modulus, int16 array [N, n_p]).

Replaces the reference's cuda_move / cuda_move_inputs / cuda_evaluate /
cuda_move_outputs (garbled_circuit_interface.h:477-736).
"""
from __future__ import annotations

from typing import Optional, Sequence

from .native import native


def _stream_handle(stream) -> int:
    if stream is None:
        try:
            import torch

            if torch.cuda.is_available():
                return int(torch.cuda.current_stream().cuda_stream)
        except Exception:
            pass
        return 0
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)


class HipEvaluator:
    def __init__(self, models: Sequence = (), device: int = 0, mfma: bool = True, profile: bool = False,
                 template=None, batch: Optional[int] = None, stream_tables: bool = False):
        """Either pass all `models` (uploaded immediately), or a `template`
        model plus a `batch` size and stream models in with `load(b, m)` so
        that host memory never holds more than one garbled model.

        stream_tables: keep the garbled tables in pinned host memory and copy each layer's tables into
        one of three rotating HBM windows one layer ahead of its use (for models or batches whose tables
        exceed the device's HBM; the tables then cross PCIe on every run)."""
        n = native()
        if n.hip_device_count() == 0:
            raise RuntimeError("dash_amd: no HIP device visible; HipEvaluator needs an MI355X (gfx950)")
        models = list(models)
        if template is None:
            if not models:
                raise ValueError("need models or a template")
            template = models[0]
        B = batch if batch is not None else len(models)
        self._h = n.HipEvaluator(template, B, device, mfma, stream_tables)
        for b, m in enumerate(models):
            self._h.load(b, m)
        if profile:
            self._h.set_profile(True)

    def load(self, b: int, model) -> None:
        self._h.load(b, model)

    def sink(self, b: int):
        """Slot b as the GPU garbler's table destination: ``GarbledCircuit(..., device=d, sink=ev.sink(b))``
        writes the tables straight into this evaluator's HBM arena, and ``load(b, gc.model)`` then copies
        only the small per-GC constants (zero-copy offline phase)."""
        return self._h.sink(b)

    def ipc_export(self) -> list:
        """IPC handles of the table arenas, ``[(layer, table, bytes per slot, handle)]``: a garbler process on the
        same node opens them (``native().IpcTables``) and garbles straight into this evaluator's slots."""
        return self._h.ipc_export()

    @property
    def batch(self) -> int:
        return self._h.batch

    @property
    def streams_tables(self) -> bool:
        return self._h.streams_tables

    def device_bytes(self) -> int:
        return self._h.device_bytes()

    def table_bytes(self) -> int:
        return self._h.table_bytes()

    def evaluate(self, inputs: Sequence, stream=None):
        """inputs: one label list per model -> list of output label lists."""
        return self._h.evaluate(list(inputs), _stream_handle(stream))

    def set_inputs(self, inputs: Sequence, stream=None):
        self._h.set_inputs(list(inputs), _stream_handle(stream))

    def set_input_cm(self, b: int, arrays) -> None:
        """Stage component-major input labels (GarbledCircuit.garble_inputs_cm) for slot b."""
        self._h.set_input_cm(b, list(arrays))

    def encode_into(self, b: int, gc, x, guarded: bool = False) -> None:
        """In-process fast path: garbler `gc` encodes x straight into the pinned staging slot b (after the
        garbler's range guard, unless the caller checked the batch itself: guarded=True)."""
        import numpy as np

        if not guarded:
            gc.check_inputs([x])
        native().encode_into(gc.garbler, np.asarray(x, dtype=np.int64).reshape(-1), self._h, b)

    def encode_device_into(self, b: int, encoder, x, stream=None) -> None:
        """Online message #1 on the device: the garbler's encoder (GarbledCircuit.device_input_encoder) writes
        W0 + x R into slot b's input activations, async on `stream` (run() on the same stream follows it).
        x of shape (n, ...) with n > 1 rows: encoder slots 0 .. n - 1 into evaluator slots b .. b + n - 1."""
        import numpy as np

        x = np.asarray(x, dtype=np.int64)
        N = encoder.input_size()
        x = x.reshape(-1) if x.size == N else x.reshape(-1, N)
        encoder.encode_into(self._h, b, x, _stream_handle(stream))

    def set_input_compressed(self, b: int, labels) -> None:
        """Stage compressed input labels ((k, N, 2) uint64, GarbledCircuit.garble_inputs_compressed)."""
        self._h.set_input_compressed(b, labels)

    def encode_compressed_into(self, b: int, gc, x, guarded: bool = False) -> None:
        """In-process fast path, wire form: the garbler writes 16-B compressed labels into slot b (after the
        garbler's range guard, unless the caller checked the batch itself: guarded=True)."""
        import numpy as np

        if not guarded:
            gc.check_inputs([x])
        native().encode_compressed_into(gc.garbler, np.asarray(x, dtype=np.int64).reshape(-1), self._h, b)

    def upload_inputs_compressed(self, stream=None) -> None:
        """H2D of the compressed slots and on-GPU decompression into the input activations."""
        self._h.upload_inputs_compressed(_stream_handle(stream))

    def fetch_outputs(self, stream=None) -> None:
        """D2H of every slot's output labels (synchronizes `stream`)."""
        self._h.fetch_outputs(_stream_handle(stream))

    def outputs_compressed(self, b: int):
        """Online message #2 of slot b in wire form: (k, n_out, 2) uint64 (after fetch_outputs)."""
        return self._h.outputs_compressed(b)

    def decode(self, b: int, gc):
        """Decode slot b's fetched outputs with the garbler's decoder (IntegrityError on tampering)."""
        return self._h.decode_into(b, gc.decoder)

    def upload_inputs(self, stream=None) -> None:
        """H2D of every staged slot (async on `stream`)."""
        self._h.upload_inputs(_stream_handle(stream))

    def run(self, stream=None):
        self._h.run(_stream_handle(stream))

    def get_outputs(self, stream=None):
        return self._h.get_outputs(_stream_handle(stream))

    def set_profile(self, on: bool = True):
        self._h.set_profile(on)

    def op_times(self):
        return self._h.op_times()

    def layer_times(self) -> dict:
        """Per-layer milliseconds of the last run (profile mode)."""
        out: dict = {}
        for name, ms in self._h.op_times():
            layer = name.split("#")[0]
            out[layer] = out.get(layer, 0.0) + ms
        return out


def hip_stream(priority: int = 0) -> int:
    """A dedicated non-blocking HIP stream (handle usable wherever a stream is accepted)."""
    return native().hip_stream_create(priority)


def hip_available() -> bool:
    try:
        return native().hip_device_count() > 0
    except Exception:
        return False
