"""Several GPUs per site (intra-site data parallelism, ``parallel.group`` module docstring): a
site input ``gpus: [0, 1]`` runs the site as 2 processes holding disjoint shards of every batch.

Checked on gloo / CPU against the one-process-per-site run on the same data: the engines' update
equals the site-level update (dSGD and PowerSGD: the mean over all ranks is the mean of the
sites' full-batch gradients; rank-dAD: each site factorises ITS gradient, formed over its
replicas first), replicas of every site stay bit-identical, and the site runtime runs end to
end with sharded splits (reference: ``datasets/icalstm/inputspec.json:6-10``, the GUI's "GPU IDs
to use, e.g. [0, 1]")."""
import os
import warnings

import pytest
import torch
import torch.nn as nn

from mp_util import run_world
from test_engines import _model


def _site_batch(site, n=12):
    g = torch.Generator().manual_seed(300 + site)
    return torch.randn(n, 12, generator=g), torch.randint(0, 3, (n,), generator=g)


def w_site_grads(grp, engine_name, cfg):
    from dinunet_implementations_amd.ops import FlatParams
    from dinunet_implementations_amd.parallel import make_engine
    m = _model()
    flat = FlatParams(m.parameters())
    eng = make_engine(engine_name, m, flat, grp, dict(cfg))
    x, y = _site_batch(grp.site)
    k, r = grp.replicas, grp.replica
    x, y = x[r::k], y[r::k]  # this replica's shard of the site's batch
    flat.zero_grad()
    with eng.step_context():
        nn.functional.cross_entropy(m(x), y).backward()
    scale = eng.reduce()
    return grp.site, grp.replica, (flat.grad * scale).clone()


@pytest.mark.parametrize("engine,cfg,tol", [
    ("dSGD", {}, 1e-6),
    ("rankDAD", {"dad_reduction_rank": 2, "dad_num_pow_iters": 6, "dad_tol": 0.0}, 1e-4),
    ("powerSGD", {"powersgd_rank": 8}, 1e-5),
])
def test_replicas_match_one_process_per_site(engine, cfg, tol):
    ref = run_world(w_site_grads, 2, engine, cfg)            # 2 sites, 1 process each
    rep = run_world(w_site_grads, 4, engine, cfg, replicas=2)  # 2 sites x 2 GPUs
    assert [(s, r) for s, r, _ in rep] == [(0, 0), (0, 1), (1, 0), (1, 1)]
    for _, _, g in rep[1:]:
        assert torch.equal(g, rep[0][2])  # every process holds the same update
    err = float((rep[0][2] - ref[0][2]).norm() / ref[0][2].norm())
    assert err < tol, err
    if engine == "rankDAD":  # the low-rank update differs from the dense mean: a real test
        dense = run_world(w_site_grads, 2, "dSGD", {})[0][2]
        assert float((ref[0][2] - dense).norm() / dense.norm()) > 10 * tol


def w_group(grp):
    t = torch.full((3,), float(grp.rank))
    grp.site_mean_(t)
    cat = grp.site_all_gather_varlen(torch.arange(grp.replica + 1).float())
    return grp.site, grp.sites, grp.replica, grp.replicas, t.tolist(), cat.tolist()


def test_site_group_fields_and_site_collectives():
    out = run_world(w_group, 6, replicas=3)
    for rank, (site, sites, rep, k, t, cat) in enumerate(out):
        assert (site, sites, rep, k) == (rank // 3, 2, rank % 3, 3)
        assert t == [float(3 * site + 1)] * 3  # mean of the site's ranks
        assert cat == [0.0, 0.0, 1.0, 0.0, 1.0, 2.0]


def test_replicas_per_site_rule_and_device_choice():
    from dinunet_implementations_amd.parallel.group import resolve_device
    from dinunet_implementations_amd.run import replicas_per_site
    two = [{"gpus": [0, 1]}, {"gpus": [2, 3]}]
    assert replicas_per_site(two, 4) == 2
    assert replicas_per_site(two, 2) == 1          # one process per site launched
    assert replicas_per_site([{"gpus": [0]}, {"gpus": [1]}], 2) == 1
    assert replicas_per_site([{"gpus": [0, 1]}, {"gpus": [2]}], 3) == 1  # not uniform
    assert replicas_per_site([{}, {}], 4, flag=2) == 2
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # the listed ids are all used: no warning
        assert resolve_device([2, 3], local_rank=3, n_devices=8, replica=1,
                              replicas=2) == torch.device("cuda", 3)
    with pytest.warns(RuntimeWarning, match="own GPU"):  # --site-gpus over one-GPU inputs
        assert resolve_device([1], local_rank=3, n_devices=8, replica=1,
                              replicas=2) == torch.device("cuda", 3)
    with pytest.warns(RuntimeWarning, match="not used"):
        assert resolve_device([2, 3, 4], local_rank=2, n_devices=8, replica=0,
                              replicas=2) == torch.device("cuda", 2)


def w_runtime(grp, data_path, out, overrides):
    from dinunet_implementations_amd.config import build_config, load_inputspec
    from dinunet_implementations_amd.runtime.site import FederatedSite
    from dinunet_implementations_amd.tasks import get_task
    specs = load_inputspec(os.path.join(data_path, "inputspec.json"))
    cfg = build_config(site_input=specs[grp.site], overrides=overrides)
    state = {"baseDirectory": os.path.join(data_path, "input", f"local{grp.site}",
                                           "simulatorRun")}
    T, D, H = get_task(cfg["task_id"])
    logs = FederatedSite(cfg, grp, T, D, H, state, out, verbose=False).run()
    return [{k: l.get(k) for k in ("test_metrics", "replica_check", "split_sizes", "num_sites",
                                "gpus_per_site", "site")} for l in logs]


def test_runtime_two_sites_two_gpus_each(fs_data_root, tmp_path):
    out = str(tmp_path)
    one = run_world(w_runtime, 2, fs_data_root, out + "/one", {"epochs": 2, "batch_size": 16})
    res = run_world(w_runtime, 4, fs_data_root, out + "/rep",
                    {"epochs": 2, "batch_size": 16, "check_replicas": True}, replicas=2)
    for r in res:
        assert r[0]["test_metrics"] == res[0][0]["test_metrics"]  # one global decision
        assert all(r[0]["replica_check"])
        assert (r[0]["num_sites"], r[0]["gpus_per_site"]) == (2, 2)
    # the replicas' shards partition each site's splits
    for s in (0, 1):
        a, b = res[2 * s][0]["split_sizes"], res[2 * s + 1][0]["split_sizes"]
        full = one[s][0]["split_sizes"]
        assert {k: a[k] + b[k] for k in a} == full
    assert os.path.exists(os.path.join(out, "rep", "local1_replica1", "FS-Classification",
                                       "fold_0", "logs.json"))
    assert os.path.exists(os.path.join(out, "rep", "remote", "FS-Classification", "fold_0",
                                       "logs.json"))
