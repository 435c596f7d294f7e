"""In-process COINSTAC simulator: N site nodes + 1 remote node over real transfer directories.

Reproduces the reference's only multi-site test harness (the COINSTAC simulator over
``datasets/*/inputspec.json``): each site gets its own ``baseDirectory`` (a
symlinked view of ``<data>/input/local<i>/simulatorRun`` plus files the remote transferred),
``transferDirectory`` and ``outputDirectory``; site transfer files are copied into the remote's
``baseDirectory/<site>/`` and remote transfer files into every site's ``baseDirectory``.
"""
from __future__ import annotations

import json
import os
import shutil
from typing import Any, Callable, Dict, List, Optional

from ..config import load_inputspec


def _fresh(d: str) -> str:
    os.makedirs(d, exist_ok=True)
    return d


def _copy_all(src: str, dst: str):
    os.makedirs(dst, exist_ok=True)
    for fn in os.listdir(src):
        p = os.path.join(src, fn)
        if os.path.isfile(p):
            shutil.copy(p, os.path.join(dst, fn))


def simulate(data_path: str, out_path: str, local_factory: Callable[[], Callable],
             remote_factory: Callable[[], Callable], max_iterations: int = 1_000_000,
             site_inputs: Optional[List[Dict[str, Any]]] = None, overrides: Optional[Dict] = None):
    specs = site_inputs or load_inputspec(os.path.join(data_path, "inputspec.json"))
    n = len(specs)
    sites = [f"local{i}" for i in range(n)]
    st = {}
    for i, s in enumerate(sites):
        base = _fresh(os.path.join(out_path, "base", s))
        src = os.path.join(data_path, "input", s, "simulatorRun")
        for fn in os.listdir(src):
            link = os.path.join(base, fn)
            if not os.path.exists(link):
                os.symlink(os.path.abspath(os.path.join(src, fn)), link)
        st[s] = {"baseDirectory": base, "transferDirectory": _fresh(os.path.join(out_path, "transfer", s)),
                 "outputDirectory": _fresh(os.path.join(out_path, "output", s, "simulatorRun")),
                 "cacheDirectory": _fresh(os.path.join(out_path, "cache", s)), "clientId": s}
    rst = {"baseDirectory": _fresh(os.path.join(out_path, "base", "remote")),
           "transferDirectory": _fresh(os.path.join(out_path, "transfer", "remote")),
           "outputDirectory": _fresh(os.path.join(out_path, "output", "remote", "simulatorRun")),
           "cacheDirectory": _fresh(os.path.join(out_path, "cache", "remote")), "clientId": "remote"}
    locals_ = {s: local_factory() for s in sites}
    remote = remote_factory()
    inputs = {s: {**specs[i], **(overrides or {})} for i, s in enumerate(sites)}
    it = 0
    outs = {s: locals_[s]({"input": inputs[s], "state": {**st[s], "iteration": it}}) for s in sites}
    while it < max_iterations:
        it += 1
        for s in sites:
            _copy_all(st[s]["transferDirectory"], os.path.join(rst["baseDirectory"], s))
        r = remote({"input": {s: outs[s]["output"] for s in sites}, "state": {**rst, "iteration": it}})
        for s in sites:
            _copy_all(rst["transferDirectory"], st[s]["baseDirectory"])
        outs = {s: locals_[s]({"input": r["output"], "state": {**st[s], "iteration": it}}) for s in sites}
        if r.get("success"):
            break
    with open(os.path.join(out_path, "simulation.json"), "w") as f:
        json.dump({"iterations": it, "sites": sites}, f)
    return it, locals_, remote
