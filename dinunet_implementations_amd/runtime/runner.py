"""Single-site harness — the ``SiteRunner`` of the reference.

``comps/fs/site_run.py:5-6`` / ``comps/icalstm/site_run.py:6-9`` construct
``SiteRunner(taks_id=..., data_path=..., mode=..., split_ratio=..., seed=..., site_index=...,
monitor_metric=..., log_header=..., batch_size=...)`` and call ``.run(Trainer, Dataset,
DataHandle)``.  The same call trains one site with no aggregator, in one process: the site's
config comes from ``data_path/inputspec.json[site_index]`` and its data from
``data_path/input/local<site_index>/simulatorRun``.  (``taks_id`` — sic — is accepted as well
as ``task_id``.)
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

from ..config import build_config, load_inputspec
from ..parallel.group import SiteGroup
from .site import FederatedSite


class SiteRunner:
    def __init__(self, taks_id: Optional[str] = None, data_path: str = ".", mode: str = "train",
                 site_index: int = 0, out_dir: Optional[str] = None, device: Optional[str] = None,
                 task_id: Optional[str] = None, **overrides: Any):
        self.task_tag = task_id or taks_id or "site"
        self.data_path = data_path
        self.site_index = int(site_index)
        self.mode = mode
        self.overrides = overrides
        self.out_dir = out_dir or os.path.join(data_path, "output")
        self.device = device

    def config(self, trainer_cls=None) -> Dict[str, Any]:
        spec_path = os.path.join(self.data_path, "inputspec.json")
        site_in = {}
        if os.path.exists(spec_path):
            specs = load_inputspec(spec_path)
            site_in = specs[self.site_index % len(specs)]
        task = site_in.get("task_id")
        if task is None and trainer_cls is not None:
            from ..tasks import TASKS
            for k, (tr, _, _) in TASKS.items():
                if issubclass(trainer_cls, tr) or trainer_cls is tr:
                    task = k
        ov = dict(self.overrides)
        ov["mode"] = str(self.mode).lower()
        if task:
            ov.setdefault("task_id", task)
        return build_config(site_input=site_in, overrides=ov)

    def state(self) -> Dict[str, Any]:
        base = os.path.join(self.data_path, "input", f"local{self.site_index}", "simulatorRun")
        if not os.path.isdir(base):
            base = self.data_path
        return {"baseDirectory": base, "clientId": f"local{self.site_index}"}

    def run(self, trainer_cls, dataset_cls, datahandle_cls):
        import torch
        cfg = self.config(trainer_cls)
        from ..parallel.group import resolve_device
        dev = torch.device(self.device) if self.device else resolve_device(cfg.get("gpus"))
        group = SiteGroup(device=dev)
        site = FederatedSite(cfg, group, trainer_cls, dataset_cls, datahandle_cls, self.state(),
                             self.out_dir, site_name=f"local{self.site_index}")
        return site.run()
