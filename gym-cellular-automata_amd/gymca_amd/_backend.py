"""Backend selection between the two builds of the C-ABI (include/gca.h).

* ``"hip"`` — libgca_hip.so, the gfx950 kernels: every device tensor, every grid above HOST_MAX_CELLS cells.
* ``"cpu"`` — libgca_cpu.so (csrc/gca_cpu.cpp), the same symbols on host pointers for the calls whose work is a
  few dozen bytes: the O(1)-per-env Move / Modify family on host arrays and whole CA steps of grids of at most
  HOST_MAX_CELLS cells (BASELINE config 1, ForestFireHelicopter5x5: a device round trip per call costs 10-100x the
  work, reference helicopter.py:220-236).
* ``"auto"`` (default) — the rule above. Device tensors never leave the device; host arrays of a large grid go to
  the GPU and fail loudly (GCAError) when there is none: nothing large ever runs on the host.

Set globally with ``set_backend`` / the ``GCA_BACKEND`` environment variable, or per operator (``backend=``).
The GPU parity tests pin ``backend="hip"`` so that they exercise the kernels, never the host build.
"""
import os

import numpy as np

from ._lib import GCAError

HOST_MAX_CELLS = 4096  # 64 x 64
_BACKENDS = ("auto", "hip", "cpu")
_default = os.environ.get("GCA_BACKEND", "auto")
if _default not in _BACKENDS:
    raise GCAError(f"GCA_BACKEND must be one of {_BACKENDS}, got {_default!r}")


def set_backend(backend):
    """Process-wide default backend ("auto", "hip" or "cpu")."""
    global _default
    if backend not in _BACKENDS:
        raise ValueError(f"backend must be one of {_BACKENDS}, got {backend!r}")
    _default = backend


def get_backend():
    return _default


def choose(backend, on_device, cells_per_env, o1=False):
    """'hip' or 'cpu' for one call. `o1`: the call's work is O(1) per env (Move / Modify)."""
    b = _default if backend is None else backend
    if b not in _BACKENDS:
        raise ValueError(f"backend must be one of {_BACKENDS}, got {b!r}")
    if b == "hip":
        return "hip"
    if b == "cpu":
        if on_device:
            raise GCAError("backend='cpu' runs on host arrays; got a device tensor")
        return "cpu"
    if on_device:
        return "hip"
    return "cpu" if (o1 or cells_per_env <= HOST_MAX_CELLS) else "hip"


def hptr(a):
    """Host address of a C-contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    if not (isinstance(a, np.ndarray) and a.flags["C_CONTIGUOUS"]):
        raise GCAError("expected a C-contiguous numpy array")
    return a.ctypes.data


class Scratch:
    """Host buffers reused across calls, with their addresses taken once (an address lookup costs about as much
    as a whole 5x5 CA step). One per operator: the reference's operators are single-threaded."""

    def __init__(self):
        self._bufs = {}

    def get(self, name, shape, dtype):
        key = (name, shape, dtype)
        hit = self._bufs.get(key)
        if hit is None:
            a = np.zeros(shape, dtype=dtype)
            hit = self._bufs[key] = (a, a.ctypes.data)
        return hit
