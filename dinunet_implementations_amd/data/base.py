"""Dataset / data-handle bases (the ``COINNDataset`` / ``COINNDataHandle`` roles).

Reference plugins subclass a torch ``Dataset`` that parses one sample per ``__getitem__`` (FS: a
CSV per subject per step, ``comps/fs/__init__.py:33-39``) in host float64.  Here the same hooks
exist (``load_index`` / ``_load_indices`` / ``__getitem__`` / ``list_files``) so a reference-style
plugin still works, but the framework calls :meth:`SiteDataset.materialize` ONCE: every sample of
the site is preprocessed into contiguous fp32 tensors that live in HBM for the whole run
(288 GB per MI355X holds any site's data), and batches are index-gathers on the device.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch


class SiteDataset(torch.utils.data.Dataset):
    def __init__(self, cache: Optional[Dict[str, Any]] = None, state: Optional[Dict[str, Any]] = None,
                 mode: str = "train", **kw):
        self.cache = cache if cache is not None else {}
        self.state = state if state is not None else {}
        self.mode = mode
        self.indices: List[Any] = []

    # reference hooks ---------------------------------------------------------------------------
    def path(self, cache_key: Optional[str] = None) -> str:
        """Site base dir (+ the file named by ``cache[cache_key]``)."""
        base = self.state.get("baseDirectory", ".")
        if cache_key is None:
            d = self.cache.get("data_dir")
            return os.path.join(base, d) if d else base
        return os.path.join(base, self.cache[cache_key])

    def load_index(self, file):
        self.indices.append(file)

    def _load_indices(self, files: Sequence[Any], **kw):
        for f in files:
            self.load_index(f)

    def add(self, files: Sequence[Any], **kw):
        self._load_indices(files, **kw)

    def __len__(self):
        return len(self.indices)

    def __getitem__(self, ix):  # pragma: no cover - subclasses
        raise NotImplementedError

    # MI355X path ------------------------------------------------------------------------------
    def materialize(self, device=None) -> Tuple[torch.Tensor, torch.Tensor]:
        """All samples as ``(inputs [N, ...] fp32, labels [N] int64)`` on ``device``."""
        xs, ys = [], []
        for i in range(len(self)):
            it = self[i]
            xs.append(torch.as_tensor(it["inputs"]).float())
            ys.append(int(torch.as_tensor(it["labels"])))
        if not xs:
            return torch.zeros(0), torch.zeros(0, dtype=torch.long)
        X = torch.stack(xs)
        y = torch.tensor(ys, dtype=torch.long)
        if device is not None:
            X, y = X.to(device), y.to(device)
        return X, y


class SiteDataHandle:
    """Lists a site's samples; the framework splits them (``data.splits``)."""

    def __init__(self, cache: Optional[Dict[str, Any]] = None, state: Optional[Dict[str, Any]] = None, **kw):
        self.cache = cache if cache is not None else {}
        self.state = state if state is not None else {}

    def list_files(self) -> List[Any]:
        base = self.state.get("baseDirectory", ".")
        return sorted(os.listdir(base))
