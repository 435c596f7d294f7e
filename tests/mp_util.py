"""Spawn a gloo process group on CPU (127.0.0.1) and collect per-rank results."""
import os
import pickle
import socket
import tempfile
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, outdir, replicas=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    os.environ.setdefault("OMP_NUM_THREADS", "2")
    import torch
    torch.set_num_threads(2)
    from dinunet_implementations_amd.parallel import init_sites, shutdown
    res = None
    grp = None
    try:
        grp = init_sites(backend="gloo", device="cpu", replicas=replicas)
        res = ("ok", fn(grp, *args))
    except Exception:  # pragma: no cover - surfaced by the parent
        res = ("err", traceback.format_exc())
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)
    # Tear down only after every rank has written its result: a rank that destroys its gloo
    # context while a peer is still sending aborts ("terminate called without an active
    # exception") in gloo's transport threads.  os._exit skips interpreter-exit destructors of
    # those threads for the same reason; the result file is already on disk.
    try:
        if grp is not None and res[0] == "ok":
            import torch.distributed as dist
            dist.barrier()
            shutdown()
    except Exception:  # pragma: no cover
        pass
    os._exit(0)


def run_world(fn, world, *args, _retry=True, replicas=1):
    """Run ``fn(grp, *args)`` on ``world`` gloo ranks (``replicas`` processes per site)."""
    try:
        return _run_world(fn, world, *args, replicas=replicas)
    except AssertionError as e:
        # free_port() -> bind is racy against other processes on the host: retry once on a
        # rendezvous port collision, never on a real failure
        if _retry and ("Address already in use" in str(e) or "EADDRINUSE" in str(e)):
            return run_world(fn, world, *args, _retry=False, replicas=replicas)
        raise


def _run_world(fn, world, *args, replicas=1):
    outdir = tempfile.mkdtemp()
    # spawn (not fork): the pytest parent has live OpenMP/autograd threads; workers must be
    # module-level functions of an importable test module
    mp.start_processes(_entry, args=(world, free_port(), fn, args, outdir, replicas), nprocs=world,
                       join=True, start_method="spawn")
    out, errs = [], []
    for r in range(world):
        with open(os.path.join(outdir, f"r{r}.pkl"), "rb") as f:
            status, val = pickle.load(f)
        if status != "ok":
            errs.append(f"rank {r} failed:\n{val}")
        out.append(val)
    if errs:
        # the root cause is usually the one that is NOT a gloo "connection closed" echo
        errs.sort(key=lambda e: "Connection closed" in e)
        raise AssertionError("\n".join(errs))
    return out
