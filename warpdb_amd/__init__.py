"""warpdb_amd -- WarpDB's query execution path on AMD Instinct MI355X.

Layers (all native, built in-tree by ``make -C warpdb_amd``):
  libwarpexec.so   C ABI (include/warpexec.h): hiprtc JIT of hand-written
                   gfx950 kernel templates; bound here by ``_warpexec``.
  libwarpdb.so     C++ host layer with the reference API (WarpDB, jit_*,
                   loaders, multi-GPU + RCCL, Arrow export).
  pywarpdb         Python module with the reference's pybind surface.

torch (when installed) is imported first so the native libraries share its
HIP runtime; torch is plumbing (device memory, streams, torch.distributed).
"""
from __future__ import annotations

import importlib

try:  # one HIP runtime per process: let torch load it first
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

__all__ = ["pywarpdb", "_warpexec", "distributed"]


def __getattr__(name):
    if name in ("pywarpdb", "_warpexec", "distributed"):
        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
