"""Exact resume: a run stopped after epoch 3 and resumed from
``checkpoint_last.pt`` reproduces the uninterrupted run's curve and weights bit for bit.

The checkpoint carries weights + optimizer, best/patience, the log history, every RNG (torch,
Python, NumPy, fused-head dropout counters), the train loader's position and the engine state
(PowerSGD error feedback and warm-started Q).  CPU/gloo, 2 sites.
"""
import json
import os

import pytest
import torch

from mp_util import run_world
from test_runtime_e2e import w_site

KEYS = ("train_log", "validation_log", "local_validation_log", "best_val_epoch")


def _logs(out, site, task):
    with open(os.path.join(out, site, task, "fold_0", "logs.json")) as f:
        return json.load(f)


def _weights(out, site, task):
    ck = torch.load(os.path.join(out, site, task, "fold_0", "checkpoint_last.pt"),
                    weights_only=True)
    return ck["models"], ck["optimizer"]


def _check_same(a_out, b_out, task):
    for site in ("local0", "local1"):
        la, lb = _logs(a_out, site, task), _logs(b_out, site, task)
        for k in KEYS:
            assert la[k] == lb[k], (site, k, la[k], lb[k])
        (ma, oa), (mb, ob) = _weights(a_out, site, task), _weights(b_out, site, task)
        for name in ma:
            for p in ma[name]:
                assert torch.equal(ma[name][p], mb[name][p]), (site, name, p)
        assert oa["step"] == ob["step"]


def test_resume_fs_dsgd_bitwise(fs_data_root, tmp_path):
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    base = {"patience": 100, "seed": 3}
    run_world(w_site, 2, fs_data_root, a, dict(base, epochs=6))
    run_world(w_site, 2, fs_data_root, b, dict(base, epochs=3))
    run_world(w_site, 2, fs_data_root, b, dict(base, epochs=6, resume=True))
    _check_same(a, b, "FS-Classification")


def test_resume_ica_powersgd_dropout_bitwise(tmp_path):
    from dinunet_implementations_amd.data.synthetic import make_ica_sites
    root = make_ica_sites(str(tmp_path / "ica"), sites=2, subjects=(24, 20), comps=8, T=60,
                          window_size=10, window_stride=10, hidden_size=16, input_size=12)
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    base = {"patience": 100, "batch_size": 8, "agg_engine": "powerSGD", "powersgd_rank": 2}
    run_world(w_site, 2, root, a, dict(base, epochs=4))
    run_world(w_site, 2, root, b, dict(base, epochs=2))
    run_world(w_site, 2, root, b, dict(base, epochs=4, resume=True))
    _check_same(a, b, "ICA-Classification")
