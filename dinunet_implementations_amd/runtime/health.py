"""Hand-off health of the persistent kernels: a timed-out in-kernel wait is an error, not data.

Two launches of a training step hand data between their own workgroups and wait with a
bounded poll (so a wedged launch cannot hang the GPU): the one-launch fused head
(``head_step.hip``: A1 / dZ1 / dZ0 hand-offs between the column workgroups and the tail) and the
one-launch rank-dAD power iteration (``lowrank.hip lr_persist_kernel``: per-layer barriers).  A
wait that gives up
records which one in a sticky error word and lets the launch finish; the data it then used is
whatever was there.  This module reads those words -- one small device-to-host copy per check --
and raises, so the site loop (``runtime.site.FederatedSite``, after every validation pass and at
the end of training) turns a silently wrong gradient into a failed run (``run.py`` exits 3).

Launch-time guards keep the waits from timing out in the first place: both launchers refuse
(falling back to their staged multi-launch forms) when their grid cannot be resident all at once
on the CUs left after a reserve for concurrent RCCL kernels (``common.h dn_fits_resident``), and
rank-dAD uses the one-launch form only when no other site process shares the GPU
(``parallel.group.SiteGroup.gpu_shared``).
"""
from __future__ import annotations

import ctypes
from typing import Iterable, List, Tuple

import torch

from ..ops import _lib

_lib.register("dn_set_spin_limit", [_lib.c_int])
_lib.register("dn_busy", [_lib.c_int, _lib.c_int, _lib.c_int, _lib.c_void_p])

# head_step.hip sync block: u32 word index of the error word (Y_ERR), codes 1 dZ1 / 2 dZ0 / 3 A1
HEAD_ERR_WORD = 160
HEAD_WAITS = {1: "dZ1 hand-off (tail -> column workgroups)",
              2: "dZ0 hand-off (column workgroups -> dX)",
              3: "A1 hand-off (column workgroups -> tail)"}


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


def _heads(modules: Iterable[torch.nn.Module]):
    for m in modules:
        for sub in m.modules():
            spec = getattr(sub, "_head", None)
            if spec is not None and getattr(spec, "_sync", None) is not None:
                yield spec


def handoff_errors(modules: Iterable[torch.nn.Module], engine=None,
                   reset: bool = True) -> List[Tuple[str, int, str]]:
    """``[(kernel, code, what)]`` of every error word that is set (and clear them, ``reset``)."""
    found = []
    for spec in _heads(modules):
        w = spec._sync[HEAD_ERR_WORD:HEAD_ERR_WORD + 1]
        code = int(w.item())
        if code:
            found.append(("head_step", code, HEAD_WAITS.get(code, "unknown wait")))
            if reset:
                w.zero_()
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
    return found


def check(modules: Iterable[torch.nn.Module], engine=None, where: str = ""):
    """Raise :class:`HandoffError` if any persistent kernel's wait timed out since the last
    check."""
    errs = handoff_errors(list(modules), engine)
    if errs:
        msg = "; ".join(f"{k} code {c:#x} ({w})" for k, c, w in errs)
        raise HandoffError(f"persistent-kernel wait timed out{(' ' + where) if where else ''}: "
                           f"{msg} -- the affected steps used incomplete data")
