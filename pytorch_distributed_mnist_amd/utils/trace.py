"""roctx ranges around the run's phases (the reference has no tracing).

Enabled with ``--trace`` or ``PDM_ROCTX=1``; a no-op otherwise or when libroctx64 cannot be
found.  Ranges nest: ``epoch N`` > ``train`` (graph replays) / ``evaluate`` / ``checkpoint``,
plus ``sampler upload`` per epoch.  View them with

    rocprofv3 --marker-trace --kernel-trace -d out -o run -- python3 multi_proc_single_gpu.py --trace ...

(markers and kernel dispatches land on one timeline; never combine with ``--pmc``).
"""
from __future__ import annotations

import contextlib
import ctypes
import ctypes.util
import os
from .. import knobs

_lib = None
_enabled = False


def _load():
    cands = [os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "libroctx64.so"),
             ctypes.util.find_library("roctx64")]
    for c in cands:
        if c:
            try:
                lib = ctypes.CDLL(c)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                return lib
            except OSError:
                continue
    return None


def enable(flag: bool = True) -> bool:
    """Turn tracing on (returns whether roctx is actually available)."""
    global _lib, _enabled
    if flag and _lib is None:
        _lib = _load()
    _enabled = bool(flag and _lib is not None)
    return _enabled


def enabled() -> bool:
    return _enabled


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    if _enabled:
        _lib.roctxRangePushA(name.encode())
        try:
            yield
        finally:
            _lib.roctxRangePop()
    else:
        yield


def mark(name: str) -> None:
    if _enabled:
        _lib.roctxMarkA(name.encode())


if knobs.get("PDM_ROCTX", "") not in ("", "0"):
    enable(True)
