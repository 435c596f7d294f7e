"""Minimal COINSTAC node runtime (``coinstac.start``, reference ``entry.py:1,5``).

If the real ``coinstac`` package is importable it is used as is.  Otherwise ``start`` serves the
two callbacks over a line-delimited JSON protocol on stdin/stdout — one request per line,
``{"type": "local" | "remote", "data": {"input": ..., "state": ...}}`` — which is what a
COINSTAC-style orchestrator (or :mod:`compat.simulator`) needs to drive a containerised node.
"""
from __future__ import annotations

import json
import sys
from typing import Callable, Dict


def start(local_fn: Callable[[Dict], Dict], remote_fn: Callable[[Dict], Dict], stdin=None, stdout=None):
    try:  # pragma: no cover - only inside a real COINSTAC image
        import coinstac  # type: ignore
        return coinstac.start(local_fn, remote_fn)
    except ImportError:
        pass
    stdin = stdin or sys.stdin
    stdout = stdout or sys.stdout
    for line in stdin:
        line = line.strip()
        if not line:
            continue
        msg = json.loads(line)
        fn = remote_fn if msg.get("type") == "remote" else local_fn
        try:
            out = fn(msg.get("data", {}))
        except Exception as e:  # report, keep serving
            out = {"error": {"message": str(e), "type": type(e).__name__}}
        stdout.write(json.dumps(out) + "\n")
        stdout.flush()
