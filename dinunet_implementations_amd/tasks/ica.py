"""ICA-Classification plugin (reference ``comps/icalstm/__init__.py``).

``ICADataset._load_indices`` loads the ``[N, C, T]`` array once (``.npy``; ``.npz`` first array
or ``data`` key — the reference's ``np.load`` of an ``.npz`` has no ``.shape``),
windows it with the reference semantics (quirk A9: ``S = int(T / W)`` windows at offset
``j * stride``) and keeps it as ONE fp32 tensor (the reference materialises float64 on the host).
``ICATrainer`` builds ``ICALstm`` from the cache (``comps/icalstm/__init__.py:45-54``) and scores
AUC on ``prob[:, 1]`` (``:64-65``).
"""
from __future__ import annotations

import csv
import os
from typing import Any, List

import numpy as np
import torch

from .. import ops
from ..data import native
from ..data.base import SiteDataHandle, SiteDataset
from ..models import ICALstm
from ..ops.reference import ica_windows
from ..runtime.trainer import NNTrainer


def load_array(path: str) -> np.ndarray:
    """``.npy`` / ``.npz`` without pickles (``allow_pickle=False``)."""
    arr = np.load(path, allow_pickle=False, mmap_mode=None)
    if isinstance(arr, np.lib.npyio.NpzFile):
        key = "data" if "data" in arr.files else arr.files[0]
        out = arr[key]
        arr.close()
        return out
    return arr


def read_lines(file: str) -> np.ndarray:
    """Reference helper (``comps/icalstm/__init__.py:12-13``): numbers, one per line, as ints."""
    with open(file) as f:
        return np.array([int(float(l.strip())) for l in f if l.strip()])


class ICADataset(SiteDataset):
    def __init__(self, **kw):
        super().__init__(**kw)
        self.data: torch.Tensor = None
        self.window_size = int(self.cache["window_size"])
        self.window_stride = int(self.cache.get("window_stride", self.window_size))
        self.temporal_size = int(self.cache["temporal_size"])
        self.num_components = int(self.cache["num_components"])

    def _load_indices(self, files, **kw):
        if self.data is None:
            shared = self.cache.get("_ica_windows_cache")
            if shared is not None:
                self.data = shared
            else:
                raw = load_array(self.path(cache_key="data_file"))
                comps = self.cache.get("components_file")
                if comps and os.path.exists(os.path.join(self.state.get("baseDirectory", "."), comps)):
                    sel = read_lines(os.path.join(self.state.get("baseDirectory", "."), comps))
                    raw = raw[:, np.asarray(sel, dtype=np.int64)]
                # C++ host runtime windows straight from fp32 / fp64 (data/native.py); the torch
                # reference (ops.reference.ica_windows) is the fallback and the test oracle
                win = native.ica_windows(raw, self.window_size, self.window_stride,
                                         self.temporal_size)
                if win is not None:
                    self.data = torch.from_numpy(win)
                else:
                    raw = torch.from_numpy(np.ascontiguousarray(raw, dtype=np.float32))
                    self.data = ica_windows(raw, self.window_size, self.window_stride,
                                            self.temporal_size)
                self.cache["_ica_windows_cache"] = self.data
        self.indices += [[int(a), int(b)] for a, b in files]

    def __getitem__(self, ix):
        data_index, y = self.indices[ix]
        return {"inputs": self.data[data_index], "labels": y}

    def materialize(self, device=None):
        if not self.indices:
            return torch.zeros(0), torch.zeros(0, dtype=torch.long)
        idx = torch.tensor([int(i[0]) for i in self.indices], dtype=torch.long)
        X = self.data.index_select(0, idx)
        y = torch.tensor([int(i[1]) for i in self.indices], dtype=torch.long)
        return (X.to(device), y.to(device)) if device is not None else (X, y)


class ICATrainer(NNTrainer):
    # the train metric ranks prob[:, 1] (comps/icalstm/__init__.py:64-65): a device-fed epoch
    # records that column of every step's output on the device (runtime.feed)
    score_column = 1

    def _init_nn_model(self):
        c = self.cache
        self.nn["net"] = ICALstm(window_size=c["window_size"], input_size=c["input_size"],
                                 hidden_size=c["hidden_size"], num_comps=c["num_components"],
                                 num_cls=c["num_class"], num_layers=c.setdefault("num_layers", 1),
                                 bidirectional=c.setdefault("bidirectional", True),
                                 norm_layer=c.get("norm_layer", "batch"))

    def forward_loss(self, x, y):
        return self.nn["net"].forward_loss(x.float(), y)

    def split_module(self):
        return self.nn["net"]  # loader batches are fp32 already: stem(x) == forward_loss's

    def score(self, out, pred):
        return out[:, 1]  # AUC on prob[:, 1] (comps/icalstm/__init__.py:64-65)


class ICADataHandle(SiteDataHandle):
    def list_files(self) -> List[Any]:
        path = os.path.join(self.state.get("baseDirectory", "."), self.cache["labels_file"])
        with open(path, newline="") as f:
            rows = [r for r in csv.reader(f) if r]
        out = []
        for r in rows:
            try:
                out.append([int(float(r[0])), int(float(r[1]))])
            except ValueError:
                continue  # header row
        return out
