"""ctypes face of the C++ host runtime library (``csrc/host/dataio.cpp`` ->
``_native/libdinunet_host.so``): parallel FreeSurfer stats ingestion, ICA windowing, exact
ROC-AUC and confusion counts.

Every function returns ``None`` when the library is not built (CPU-only checkouts without a C++
toolchain); callers then use the Python reference implementation, which is also the oracle the
tests hold the native code to.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_native", "libdinunet_host.so")

_lib: Optional[ctypes.CDLL] = None
_tried = False
_lock = threading.Lock()

_P, _L, _I, _D = ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_double


def _load() -> Optional[ctypes.CDLL]:
    global _lib, _tried
    if _lib is not None or _tried:
        return _lib
    with _lock:
        if _lib is not None or _tried:
            return _lib
        _tried = True
        if os.environ.get("DINUNET_HOST_NATIVE", "1") == "0":
            return None
        if not os.path.exists(LIB_PATH) and os.environ.get("DINUNET_AUTOBUILD", "1") == "1":
            try:
                from ..csrc import build
                build.build_host(verbose=False)
            except Exception:  # noqa: BLE001 - fall back to Python
                return None
        if not os.path.exists(LIB_PATH):
            return None
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError:
            return None
        lib.dnh_fs_load.argtypes = [ctypes.POINTER(ctypes.c_char_p), _L, _I, _P, _I]
        lib.dnh_fs_load.restype = _L
        lib.dnh_ica_windows.argtypes = [_P, _I, _L, _I, _I, _I, _I, _I, _P, _L, _P, _I]
        lib.dnh_ica_windows.restype = _I
        lib.dnh_roc_auc.argtypes = [_P, _P, _L]
        lib.dnh_roc_auc.restype = _D
        lib.dnh_confusion2.argtypes = [_P, _P, _L, _P]
        lib.dnh_confusion2.restype = _I
        _lib = lib
        return _lib


def available() -> bool:
    return _load() is not None


def _threads() -> int:
    return int(os.environ.get("DINUNET_HOST_THREADS", "0"))


def fs_load(paths: Sequence[str], nfeat: int) -> Optional[np.ndarray]:
    """``[n, nfeat]`` fp32, each row divided by its maximum (reference quirk A8)."""
    L = _load()
    if L is None:
        return None
    n = len(paths)
    out = np.empty((n, nfeat), dtype=np.float32)
    if n == 0:
        return out
    arr = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
    rc = L.dnh_fs_load(arr, n, int(nfeat), out.ctypes.data, _threads())
    if rc != 0:
        idx, kind = divmod(int(rc) - 1, 4)
        what = {1: "cannot be read", 2: "has a malformed value", 3: f"has fewer than {nfeat} values"}
        raise ValueError(f"FreeSurfer stats file {paths[idx]!r} {what.get(kind, 'failed')}")
    return out


def ica_windows(src: np.ndarray, window_size: int, window_stride: int, temporal_size: int,
                rows: Optional[np.ndarray] = None) -> Optional[np.ndarray]:
    """``src[N, C, T]`` (fp32 / fp64) -> ``[n, S, C, W]`` fp32 for ``rows`` (all when None),
    ``S = int(temporal_size / W)`` windows at offset ``j * stride`` (reference quirk A9)."""
    L = _load()
    if L is None:
        return None
    if src.dtype not in (np.float32, np.float64):
        src = src.astype(np.float32)
    src = np.ascontiguousarray(src)
    N, C, T = src.shape
    S = int(temporal_size / window_size)
    if rows is None:
        n, rp = N, None
    else:
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        n, rp = rows.size, rows.ctypes.data
    out = np.empty((n, S, C, window_size), dtype=np.float32)
    rc = L.dnh_ica_windows(src.ctypes.data, int(src.dtype == np.float64), N, C, T,
                           int(window_size), int(window_stride), int(temporal_size), rp, n,
                           out.ctypes.data, _threads())
    if rc == 2:
        raise ValueError(f"windowing needs {(S - 1) * window_stride + window_size} time points "
                         f"(data has {T}) or a row index is out of range")
    if rc != 0:
        raise ValueError("bad ICA windowing arguments")
    return out


def roc_auc(scores: np.ndarray, labels: np.ndarray) -> Optional[float]:
    L = _load()
    if L is None:
        return None
    s = np.ascontiguousarray(np.asarray(scores, dtype=np.float64).ravel())
    y = np.ascontiguousarray(np.asarray(labels).ravel().astype(np.int64))
    return float(L.dnh_roc_auc(s.ctypes.data, y.ctypes.data, s.size))


def confusion2(pred: np.ndarray, labels: np.ndarray) -> Optional[np.ndarray]:
    """``[tn, fp, fn, tp]`` of binary hard predictions."""
    L = _load()
    if L is None:
        return None
    p = np.ascontiguousarray(np.asarray(pred).ravel().astype(np.int64))
    y = np.ascontiguousarray(np.asarray(labels).ravel().astype(np.int64))
    out = np.zeros(4, dtype=np.int64)
    L.dnh_confusion2(p.ctypes.data, y.ctypes.data, p.size, out.ctypes.data)
    return out
