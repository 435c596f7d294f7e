"""COINSTAC compatibility: file-transport simulator with the reference entry contract (CPU)."""
import io
import json
import os

import pytest
import torch


@pytest.mark.parametrize("engine", ["dSGD", "rankDAD", "powerSGD"])
def test_simulator_all_engines(fs_data_root, tmp_path, engine):
    from dinunet_implementations_amd.compat.nodes import LocalNode, RemoteNode
    from dinunet_implementations_amd.compat.simulator import simulate
    it, locs, rem = simulate(fs_data_root, str(tmp_path), lambda: LocalNode(device="cpu"), RemoteNode,
                             overrides={"epochs": 2, "agg_engine": engine})
    ws = [locs[s].trainer.flat.data for s in sorted(locs)]
    assert all(torch.equal(w, ws[0]) for w in ws)  # replicas identical through files
    r = json.load(open(os.path.join(str(tmp_path), "output", "remote", "simulatorRun",
                                    "FS-Classification", "fold_0", "logs.json")))
    assert r["agg_engine"] == engine and len(r["test_metrics"]) == 6
    assert "remote_iter_duration" in r
    site_log = os.path.join(str(tmp_path), "output", "local1", "simulatorRun", "FS-Classification",
                            "fold_0", "logs.json")
    assert "local_iter_duration" in json.load(open(site_log))
    assert os.path.exists(os.path.join(str(tmp_path), "transfer", "remote",
                                       "FS-Classification_fold_0_results.zip"))


def test_simulator_pretrain(fs_data_root, tmp_path):
    from dinunet_implementations_amd.compat.nodes import LocalNode, RemoteNode
    from dinunet_implementations_amd.compat.simulator import simulate
    it, locs, rem = simulate(fs_data_root, str(tmp_path), lambda: LocalNode(device="cpu"), RemoteNode,
                             overrides={"epochs": 1, "pretrain": True,
                                        "pretrain_args": {"epochs": 1, "learning_rate": 1e-3,
                                                          "batch_size": 16, "patience": 3}})
    assert rem.pretrain_site == "local4"  # 120 subjects: the largest site


def test_reference_entry_callbacks_and_stdio(fs_data_root, tmp_path):
    """local.run / remote.run keep the reference's module-level callback contract."""
    import importlib
    import local as site_cb
    import remote as remote_cb
    importlib.reload(site_cb)
    importlib.reload(remote_cb)
    from dinunet_implementations_amd.compat.coinstac import start
    from dinunet_implementations_amd.compat.simulator import simulate
    it, locs, rem = simulate(fs_data_root, str(tmp_path), lambda: (lambda d: site_cb.run(d)),
                             lambda: (lambda d: remote_cb.run(d)),
                             overrides={"epochs": 1}, max_iterations=3)
    assert "cumulative_total_duration" in site_cb.CACHE and it == 3
    buf = io.StringIO()
    start(lambda d: {"output": {"echo": d["input"]}}, lambda d: {"output": "r"},
          stdin=io.StringIO('{"type": "local", "data": {"input": 1}}\n{"type": "remote"}\n'),
          stdout=buf)
    lines = [json.loads(l) for l in buf.getvalue().splitlines()]
    assert lines == [{"output": {"echo": 1}}, {"output": "r"}]


def test_simulator_validation_epochs(fs_data_root, tmp_path):
    """The remote validates every `validation_epochs` epochs (compspec.json:149-160), like the
    collective runtime; training still runs every epoch and ends with a test."""
    from dinunet_implementations_amd.compat.nodes import LocalNode, RemoteNode
    from dinunet_implementations_amd.compat.simulator import simulate
    it, locs, rem = simulate(fs_data_root, str(tmp_path), lambda: LocalNode(device="cpu"), RemoteNode,
                             overrides={"epochs": 5, "validation_epochs": 2, "patience": 100})
    r = json.load(open(os.path.join(str(tmp_path), "output", "remote", "simulatorRun",
                                    "FS-Classification", "fold_0", "logs.json")))
    assert len(r["validation_log"]) == 2           # epochs 2 and 4
    assert r["best_val_epoch"] in (2, 4)
    assert len(r["cumulative_total_duration"]) == 5  # every epoch ends once
    site = json.load(open(os.path.join(str(tmp_path), "output", "local0", "simulatorRun",
                                       "FS-Classification", "fold_0", "logs.json")))
    assert len(site["train_log"]) == 5 and len(site["validation_log"]) == 2
    ws = [locs[s].trainer.flat.data for s in sorted(locs)]
    assert all(torch.equal(w, ws[0]) for w in ws)
