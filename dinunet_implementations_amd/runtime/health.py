"""Hand-off health of the kernels that wait: a timed-out in-kernel wait is an error, not data.

Two kinds of launches wait with a bounded poll (so a wedged launch cannot hang the GPU): the
one-launch rank-dAD power iteration (``lowrank.hip lr_persist_kernel``: per-layer barriers
between its own workgroups) and the peer exchange (``peer.hip``: flags written by the other
sites' launches; a dead or hung peer).  A wait that gives up records which one in a sticky error
word and lets the launch finish; the data it then used is whatever was there.  This module reads
those words -- one small device-to-host copy per check -- and raises, so the site loop
(``runtime.site.FederatedSite``, after every validation pass and at the end of training) turns a
silently wrong gradient into a failed run (``run.py`` exits 3).

Launch-time guards keep the waits from timing out in the first place: the power iteration
refuses (falling back to its staged multi-launch form) when its grid cannot be resident all at
once on the CUs left after a reserve for concurrent RCCL kernels (``common.h
dn_fits_resident``), and runs only when no other site process shares the GPU
(``parallel.group.SiteGroup.gpu_shared``); with a shared GPU the peer exchange's waits become
one-workgroup launches of their own (``parallel.peer``).  (The round-4 hand-off head, whose
waits this module also watched, is folded into the replicated head, which waits on nothing.)
"""
from __future__ import annotations

import ctypes
from typing import Iterable, List, Tuple

import torch

from ..ops import _lib

_lib.register("dn_set_spin_limit", [_lib.c_int])
_lib.register("dn_busy", [_lib.c_int, _lib.c_int, _lib.c_int, _lib.c_void_p])

class HandoffError(RuntimeError):
    """A persistent kernel's in-kernel wait timed out: that step's results are not valid."""


def set_spin_limit(polls: int):
    """Poll limit of every in-kernel wait (< 0: the kernels' defaults; 0: give up at once, the
    negative control of :func:`check`)."""
    _lib.call("dn_set_spin_limit", int(polls))


def occupy_cus(blocks: int = 64, us: int = 2000, threads: int = 256):
    """Hold ``blocks`` CUs (one spinning workgroup each, ``us`` microseconds, at most 100 ms) on
    the CURRENT stream: the footprint of RCCL's channel kernels during a collective.  Tests launch
    it on a side stream beside the persistent kernels, which reserve ``DN_RESERVE_CUS`` (64) CUs
    for exactly these (csrc/kernels/common.h)."""
    _lib.call("dn_busy", int(blocks), int(threads), int(us), _lib.stream())


def handoff_errors(modules: Iterable[torch.nn.Module], engine=None,
                   reset: bool = True) -> List[Tuple[str, int, str]]:
    """``[(kernel, code, what)]`` of every error word that is set (and clear them, ``reset``).
    ``modules`` is accepted for the callers' signature (no module-owned word is left)."""
    found = []
    table = getattr(engine, "_table", None) if engine is not None else None
    sync = getattr(table, "_persist", None)
    if sync is not None:
        w = sync[2][-1:]
        code = int(w.item())
        if code:
            phase = {1: "P / Gram barrier", 2: "Q barrier"}.get(code >> 8, "barrier")
            found.append(("lr_persist", code, f"layer {code & 0xff} {phase}"))
            if reset:
                w.zero_()
    if engine is None or getattr(engine, "peer", False):
        from ..parallel import peer as _peer
        for site, code, what in _peer.errors(reset):
            found.append(("peer_exchange", code, f"site {site}: {what}"))
    return found


def check(modules: Iterable[torch.nn.Module], engine=None, where: str = ""):
    """Raise :class:`HandoffError` if any persistent kernel's wait timed out since the last
    check."""
    errs = handoff_errors(list(modules), engine)
    if errs:
        msg = "; ".join(f"{k} code {c:#x} ({w})" for k, c, w in errs)
        raise HandoffError(f"persistent-kernel wait timed out{(' ' + where) if where else ''}: "
                           f"{msg} -- the affected steps used incomplete data")
