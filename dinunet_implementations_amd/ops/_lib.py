"""ctypes binding of the in-tree gfx950 kernel library (``_native/libdinunet_kernels.so``).

The library exposes a C ABI of raw device pointers + ``hipStream_t``.  It is loaded only after
``import torch`` so it shares torch's HIP runtime (same SONAME ``libamdhip64.so.7``).

Policy: on a machine with a GPU, every fused op REQUIRES this library; a missing or stale build
raises instead of silently running an eager fallback (``DINUNET_REQUIRE_NATIVE=0`` relaxes this
for debugging only).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_native", "libdinunet_kernels.so")
# tuning: a variant build of the same sources (tools/build_variant.py) in place of the default
LIB_PATH = os.environ.get("DINUNET_KERNEL_LIB") or LIB_PATH

_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()
_load_error: Optional[str] = None

c_void_p, c_int, c_long, c_float = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float
c_double = ctypes.c_double

# name -> argtypes (restype is always int status)
_SIGS = {
    "dn_lstm_padded_hidden": [c_int],
    "dn_lstm_pack": [c_void_p] * 8 + [c_int, c_int, c_int] + [c_void_p] * 4
                    + [c_int, c_void_p, c_void_p, c_void_p] + [c_void_p],
    # (the LSTM launchers are registered with their signatures by ops.lstm)
}


def register(name: str, argtypes):
    _SIGS[name] = argtypes
    if _lib is not None and hasattr(_lib, name):
        fn = getattr(_lib, name)
        fn.argtypes = argtypes
        fn.restype = c_int


def _load() -> Optional[ctypes.CDLL]:
    global _lib, _load_error
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH) and os.environ.get("DINUNET_AUTOBUILD", "1") == "1":
            try:
                from ..csrc import build
                build.build_kernels(verbose=False)
            except Exception as e:  # pragma: no cover - reported below
                _load_error = f"auto-build failed: {e}"
        if not os.path.exists(LIB_PATH):
            _load_error = _load_error or f"{LIB_PATH} not built (python -m dinunet_implementations_amd.csrc.build)"
            return None
        if os.environ.get("DINUNET_ALLOW_STALE", "0") != "1":
            # a library older than its sources has an older C ABI: calling it through the
            # current signatures passes arguments in the wrong slots (e.g. a null stream)
            try:
                from ..csrc import build
                stale = build.kernels_stale()
            except Exception:  # pragma: no cover
                stale = False
            if stale:
                _load_error = (f"{LIB_PATH} is stale: the kernel sources changed since it was built "
                               "(python -m dinunet_implementations_amd.csrc.build)")
                return None
        try:
            lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            _load_error = str(e)
            return None
        for name, argtypes in _SIGS.items():
            if hasattr(lib, name):
                fn = getattr(lib, name)
                fn.argtypes = argtypes
                fn.restype = c_int
        _lib = lib
        return _lib


def native_available() -> bool:
    return _load() is not None


def lib() -> ctypes.CDLL:
    L = _load()
    if L is None:
        raise RuntimeError(f"dinunet native kernels unavailable: {_load_error}")
    return L


def require_native() -> bool:
    return os.environ.get("DINUNET_REQUIRE_NATIVE", "1") != "0"


_SYNC_CHECK = os.environ.get("DINUNET_SYNC_CHECK", "0") == "1"


def call(name: str, *args) -> None:
    """Call a native launcher; raise on a non-zero status.  With ``DINUNET_SYNC_CHECK=1`` every
    launch is followed by a device synchronize so an asynchronous fault is attributed to the
    kernel that caused it (the HIP_LAUNCH_BLOCKING debug mode of SURVEY.md §5.2)."""
    fn = getattr(lib(), name)
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with status {rc}")
    if _SYNC_CHECK and torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:  # pragma: no cover - GPU fault path
            raise RuntimeError(f"{name}: device error after launch: {e}") from e


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream
