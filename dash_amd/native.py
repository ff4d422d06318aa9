"""Loader for the in-tree native extension ``_dash_native``.

torch is imported first so that the extension binds to the HIP runtime torch
already loaded (both carry the SONAME ``libamdhip64.so.7``): one HIP runtime
per process, device pointers interchangeable with torch tensors.
"""
from __future__ import annotations

import os

try:  # noqa: SIM105 - torch is optional for CPU-only tooling
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    torch = None  # type: ignore

_mod = None


def load():
    global _mod
    if _mod is not None:
        return _mod
    try:
        from . import _dash_native as m  # type: ignore
    except ImportError as e:  # pragma: no cover - build missing
        if os.environ.get("DASH_AUTOBUILD", "1") == "1":
            from . import _build

            _build.build()
            from . import _dash_native as m  # type: ignore
        else:
            raise ImportError("dash_amd native extension missing; run `python -m dash_amd._build`") from e
    _mod = m
    return m


def native():
    return load()
