"""Site runtime end to end on the GPU: ICA (fused LSTM kernels, HIP-graph train step) and FS
(fused MLP head) through train -> validation -> early-stopping bookkeeping -> test -> logs, and
once more with a 1-rank RCCL group that takes every collective code path (broadcast, bucketed
all-reduce between split graphs, variable-length metric gathers, barriers)."""
import json
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _run_site(root, out, overrides, group=None):
    from dinunet_implementations_amd.config import build_config, load_inputspec
    from dinunet_implementations_amd.parallel.group import SiteGroup
    from dinunet_implementations_amd.runtime.site import FederatedSite
    from dinunet_implementations_amd.tasks import get_task
    specs = load_inputspec(os.path.join(root, "inputspec.json"))
    cfg = build_config(site_input=specs[0], overrides=overrides)
    state = {"baseDirectory": os.path.join(root, "input", "local0", "simulatorRun")}
    T, D, H = get_task(cfg["task_id"])
    grp = group or SiteGroup(device=torch.device("cuda", 0))
    return FederatedSite(cfg, grp, T, D, H, state, out, verbose=False).run()


def _ica_root(tmp_path):
    from dinunet_implementations_amd.data.synthetic import make_ica_sites
    return make_ica_sites(str(tmp_path / "ica"), sites=1, subjects=(64,), comps=16, T=120,
                          window_size=10, window_stride=10, hidden_size=64, input_size=32)


@pytest.mark.parametrize("engine", ["dSGD", "rankDAD", "powerSGD"])
def test_ica_site_on_gpu(tmp_path, engine):
    root = _ica_root(tmp_path)
    out = str(tmp_path / "out")
    logs = _run_site(root, out, {"epochs": 3, "batch_size": 8, "agg_engine": engine,
                                 "dad_reduction_rank": 4})
    lg = logs[0]
    assert len(lg["train_log"]) == 3
    tm = lg["test_metrics"]
    assert tm and all(v == v for v in (tm if isinstance(tm, list) else tm.values())
                      if isinstance(v, float))
    found = [f for _, _, fs in os.walk(out) for f in fs]
    assert "logs.json" in found and "test_metrics.csv" in found


def test_fs_site_on_gpu(fs_data_root, tmp_path):
    logs = _run_site(fs_data_root, str(tmp_path / "out"), {"epochs": 3, "batch_size": 16})
    assert len(logs[0]["train_log"]) == 3 and logs[0]["test_metrics"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_ica_site_collective_paths_over_rccl(tmp_path):
    from test_step_gpu import _OneRankGroup
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        root = _ica_root(tmp_path)
        out = str(tmp_path / "out")
        logs = _run_site(root, out, {"epochs": 2, "batch_size": 8},
                         group=_OneRankGroup(dist.group.WORLD))
        assert len(logs[0]["train_log"]) == 2 and logs[0]["test_metrics"]
        with open(next(os.path.join(d, f) for d, _, fs in os.walk(out) for f in fs
                       if f == "logs.json")) as f:
            assert "best_val_epoch" in json.load(f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("li", [1, 2])
def test_ica_site_device_feed_matches_host_feed(tmp_path, li):
    """The production site loop trains its epochs device-fed (runtime.feed: HBM-resident bf16
    split, K-step graphs, train records on the device) and logs what the per-step host loop
    logs: same train loss / AUC per epoch, same validation curve, same test metrics; also with
    gradient accumulation (local_iterations = 2: whole accumulated steps per replay)."""
    root = _ica_root(tmp_path)
    ov = {"epochs": 3, "batch_size": 8, "seed": 3, "local_iterations": li}
    dev = _run_site(root, str(tmp_path / "dev"), dict(ov, device_feed=True))[0]
    host = _run_site(root, str(tmp_path / "host"), dict(ov, device_feed=False))[0]
    assert dev.get("feed") == "device" and "feed" not in host
    for a, b in zip(dev["train_log"], host["train_log"]):
        assert abs(a[0] - b[0]) < 2e-4 and abs(a[1] - b[1]) < 2e-3, (dev["train_log"], host["train_log"])
    for a, b in zip(dev["validation_log"], host["validation_log"]):
        assert abs(a[0] - b[0]) < 2e-4 and abs(a[1] - b[1]) < 2e-3
    assert len(dev["samples_per_sec"]) == 3


def test_fs_site_device_feed_matches_host_feed(fs_data_root, tmp_path):
    """The FS task trains device-fed too (fp32 features resident, hard-label train scores from
    the predicted class): the same logs as the per-step host loop."""
    ov = {"epochs": 3, "batch_size": 16, "seed": 3}
    dev = _run_site(fs_data_root, str(tmp_path / "dev"), dict(ov, device_feed=True))[0]
    host = _run_site(fs_data_root, str(tmp_path / "host"), dict(ov, device_feed=False))[0]
    assert dev.get("feed") == "device" and "feed" not in host
    for a, b in zip(dev["train_log"], host["train_log"]):
        assert abs(a[0] - b[0]) < 2e-4 and abs(a[1] - b[1]) < 2e-3, (dev["train_log"], host["train_log"])
    for a, b in zip(dev["validation_log"], host["validation_log"]):
        assert abs(a[0] - b[0]) < 2e-4 and abs(a[1] - b[1]) < 2e-3


@pytest.mark.parametrize("engine", ["dSGD", "rankDAD"])
def test_ica_two_sites_two_gpus_each_on_one_gpu(tmp_path, engine):
    """Several GPUs per site (``run.py --site-gpus 2``, parallel.group): 2 sites x 2 processes
    -- launched as the driver launches a node, rehearsed on the one GPU over gloo -- train the ICA
    model with the fused kernels on sharded splits; every process ends with bit-identical
    parameters (check_replicas), one global test decision, logs per site and replica."""
    import subprocess
    import sys
    from dinunet_implementations_amd.data.synthetic import make_ica_sites
    root = make_ica_sites(str(tmp_path / "ica"), sites=2, subjects=(64, 64), comps=16, T=120,
                          window_size=10, window_stride=10, hidden_size=64, input_size=32)
    out = str(tmp_path / "out")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DINUNET_BACKEND="gloo", PYTHONPATH=repo, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           "4", "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m",
           "dinunet_implementations_amd.run", "--data-path", root, "--out", out,
           "--site-gpus", "2", "--set", "epochs=2", "--set", "batch_size=8", "--set",
           f"agg_engine={engine}", "--set", "dad_reduction_rank=4", "--set",
           "check_replicas=true"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-4000:]
    logs = {}
    for name in ("local0", "local0_replica1", "local1", "local1_replica1", "remote"):
        p = os.path.join(out, name)
        f = next(os.path.join(d, x) for d, _, fs in os.walk(p) for x in fs if x == "logs.json")
        with open(f) as fh:
            logs[name] = json.load(fh)
    tm = {n: l["test_metrics"] for n, l in logs.items()}
    assert len({json.dumps(v) for v in tm.values()}) == 1, tm  # one global decision
    for n in ("local0", "local0_replica1", "local1", "local1_replica1"):
        assert all(logs[n]["replica_check"]), n
        assert logs[n]["gpus_per_site"] == 2 and logs[n]["num_sites"] == 2
    assert logs["local0"]["split_sizes"]["train"] + logs["local0_replica1"]["split_sizes"]["train"] > 0
