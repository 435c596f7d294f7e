"""Launch a decentralized run: one process per site (GPU), e.g.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m dinunet_implementations_amd.run --data-path datasets/icalstm --out out/

Rank r is site ``local<r>``: its inputs are ``inputspec.json[r]`` (the simulator convention of
``datasets/*/inputspec.json``, one object per site) and its data directory is
``<data-path>/input/local<r>/simulatorRun``.  ``--set key=value`` overrides any config key
(JSON-parsed values), e.g. ``--set agg_engine=rankDAD --set epochs=5``.
Without a launcher it runs a single site on one device.

A site input listing several GPUs (``"gpus": [0, 1]`` in every site's input, or ``--site-gpus
k``) runs each site as ``k`` data-parallel processes: launch ``sites * k`` processes; rank r is
replica ``r % k`` of site ``r // k`` (``parallel.group`` module docstring).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import traceback
from typing import Any, Dict, List


def parse_sets(items: List[str]) -> Dict[str, Any]:
    out = {}
    for it in items or []:
        k, _, v = it.partition("=")
        try:
            out[k] = json.loads(v)
        except json.JSONDecodeError:
            out[k] = v
    return out


def apply_collective_plan(cfg: Dict[str, Any]):
    """RCCL algorithm / protocol for the xGMI mesh from the config (``rccl_algo``,
    ``rccl_proto``; see README "Collective plan"), exported before the process group is
    created.  An explicit NCCL_ALGO / NCCL_PROTO in the environment wins."""
    for key, env in (("rccl_algo", "NCCL_ALGO"), ("rccl_proto", "NCCL_PROTO")):
        v = cfg.get(key)
        if v:
            os.environ.setdefault(env, str(v))


def replicas_per_site(specs: List[Dict[str, Any]], world: int, flag=None) -> int:
    """Processes per site: ``--site-gpus`` when given, else the common length of every site
    input's ``gpus`` list when that length is > 1 and the launch has exactly ``len(specs) *
    length`` processes; 1 otherwise (one process = one site)."""
    if flag:
        return max(1, int(flag))
    lens = set()
    for sp in specs:
        v = sp.get("gpus", {})
        v = v.get("value") if isinstance(v, dict) else v
        if v is None:
            return 1
        lens.add(len(v) if isinstance(v, (list, tuple)) else 1)
    if len(lens) == 1:
        k = lens.pop()
        if k > 1 and world == len(specs) * k:
            return k
    return 1


def site_gpus(cfg: Dict[str, Any], rank: int, n_specs: int, device=None):
    """The ``gpus`` pin of this rank's site input, when that input is this rank's own: with more
    ranks than inputspec entries, rank r reuses ``specs[r % n]`` and its GPU ids name ANOTHER
    site's GPU, so those ranks take their own GPU (``LOCAL_RANK``) instead.  ``gpus = []`` (the
    reference's CPU-only FreeSurfer sites, ``datasets/test_fsl/inputspec.json:15-17``) keeps the
    CPU unless ``--device`` says otherwise, and says so."""
    gpus = cfg.get("gpus")
    if rank >= n_specs:
        return None
    if gpus is not None and len(list(gpus if not isinstance(gpus, int) else [gpus])) == 0 \
            and device in (None, "", "auto"):
        print(f"[local{rank}] site input gpus=[]: this site runs on the CPU "
              f"(--device cuda overrides)", file=sys.stderr, flush=True)
    return gpus


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--data-path", required=True)
    ap.add_argument("--out", default=None)
    ap.add_argument("--device", default=None, choices=[None, "cpu", "cuda"])
    ap.add_argument("--set", action="append", default=[])
    ap.add_argument("--site-gpus", type=int, default=None,
                    help="processes (GPUs) per site; default: the sites' common gpus length")
    a = ap.parse_args(argv)
    from .config import build_config, load_inputspec
    from .parallel import init_sites, shutdown
    from .runtime.site import FederatedSite
    from .tasks import get_task

    specs = load_inputspec(os.path.join(a.data_path, "inputspec.json"))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    k = replicas_per_site(specs, world, a.site_gpus)
    site = rank // k
    site_in = specs[site % len(specs)]
    cfg = build_config(site_input=site_in, overrides=parse_sets(a.set))
    apply_collective_plan(cfg)  # before the communicator exists
    grp = init_sites(device=a.device, timeout_s=cfg.get("collective_timeout_s"),
                     gpus=site_gpus(cfg, site, len(specs), a.device), replicas=k)
    base = os.path.join(a.data_path, "input", f"local{grp.site}", "simulatorRun")
    if not os.path.isdir(base):
        base = os.path.join(a.data_path, "input", f"local{grp.site % len(specs)}", "simulatorRun")
    state = {"baseDirectory": base, "clientId": f"local{grp.site}"}
    out = a.out or os.path.join(a.data_path, "output")
    T, D, H = get_task(cfg["task_id"])
    try:
        FederatedSite(cfg, grp, T, D, H, state, out, site_name=f"local{grp.site}").run()
    except Exception as e:  # a peer site died / timed out, or this site failed
        # report and leave without tearing the process group down: a destroy that waits on a
        # dead peer would hang this survivor too
        # the traceback tells a local bug (shape error, kernel status) from a dead peer
        traceback.print_exc(file=sys.stderr)
        print(f"[local{grp.site}] site failure ({type(e).__name__}): {e}", file=sys.stderr,
              flush=True)
        sys.stdout.flush()
        os._exit(3)
    shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
