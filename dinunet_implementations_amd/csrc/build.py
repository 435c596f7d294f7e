"""Build the gfx950 kernel library in-tree.

Every ``csrc/kernels/*.hip`` file is compiled with ``hipcc --offload-arch=gfx950`` and linked
into ONE shared object, ``dinunet_implementations_amd/_native/libdinunet_kernels.so``, exposing a
plain C ABI (raw device pointers + ``hipStream_t``).  Python binds it with ``ctypes`` *after*
``import torch``, so the library resolves ``libamdhip64.so.7`` to the runtime torch already
loaded: one HIP runtime, one set of streams, graph capture works.

The host-side runtime pieces (``csrc/host/*.cpp``: data preprocessing, metric kernels for the
CPU) are compiled into ``libdinunet_host.so`` with the system C++ compiler.

Usage: ``python -m dinunet_implementations_amd.csrc.build [--force] [--jobs N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
OUT_DIR = os.path.join(PKG, "_native")
KERNEL_LIB = os.path.join(OUT_DIR, "libdinunet_kernels.so")
HOST_LIB = os.path.join(OUT_DIR, "libdinunet_host.so")
ARCH = os.environ.get("DINUNET_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", shutil.which("g++") or "c++")

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=fast",
             "-munsafe-fp-atomics", "-fno-slp-vectorize", "-Wno-unused-result"]


# per-file code-generation flags: the low-rank kernels' fp64 / f32 MFMA accumulators stay in
# VGPRs (the AGPR form made hipcc copy every loop-carried accumulator AGPR <-> VGPR each
# iteration of the Gram loop: 19k -> see profiles/r2_lowrank_stamps.txt)
FILE_FLAGS = {"lowrank.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}


def _sources(kind: str):
    if kind == "hip":
        return sorted(glob.glob(os.path.join(HERE, "kernels", "*.hip")))
    return sorted(glob.glob(os.path.join(HERE, "host", "*.cpp")))


def _digest(paths, extra: str) -> str:
    h = hashlib.sha256(extra.encode())
    deps = set(paths)
    for d in ("kernels", "host"):
        deps.update(glob.glob(os.path.join(HERE, d, "*.h")))
    for p in sorted(deps):
        with open(p, "rb") as f:
            # relative names: the digest must not depend on where the tree lives (the GPU box
            # runs a copy at another path and checks the library against its sources)
            h.update(os.path.relpath(p, HERE).encode())
            h.update(f.read())
    return h.hexdigest()


def _stamp_ok(lib: str, digest: str) -> bool:
    stamp = lib + ".sha256"
    return os.path.exists(lib) and os.path.exists(stamp) and open(stamp).read().strip() == digest


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stderr[-6000:]}")
    return r


def _kernel_digest() -> str:
    return _digest(_sources("hip"), " ".join(HIP_FLAGS) + ARCH + repr(sorted(FILE_FLAGS.items())))


def kernels_stale() -> bool:
    """True when the built kernel library does not match the kernel sources next to it (a build
    that failed after a source edit leaves the previous library in place)."""
    if not _sources("hip"):
        return False  # sources stripped: nothing to compare against
    return not _stamp_ok(KERNEL_LIB, _kernel_digest())


def build_kernels(force: bool = False, jobs: int = 4, verbose: bool = True) -> str:
    srcs = _sources("hip")
    os.makedirs(OUT_DIR, exist_ok=True)
    digest = _kernel_digest()
    if not force and _stamp_ok(KERNEL_LIB, digest):
        return KERNEL_LIB
    objdir = os.path.join(OUT_DIR, "obj")
    os.makedirs(objdir, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        flags = [*HIP_FLAGS, *FILE_FLAGS.get(os.path.basename(src), [])]
        # per-object stamp (source + every header + flags): an edit recompiles only its file
        od = _digest([src], " ".join(flags) + ARCH)
        if not force and _stamp_ok(obj, od):
            return obj
        _run([HIPCC, *flags, "-I", os.path.join(HERE, "kernels"), "-c", src, "-o", obj])
        with open(obj + ".sha256", "w") as f:
            f.write(od)
        if verbose:
            print(f"[build] {os.path.relpath(src, PKG)}", flush=True)
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = KERNEL_LIB + ".tmp"
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp])
    os.replace(tmp, KERNEL_LIB)
    with open(KERNEL_LIB + ".sha256", "w") as f:
        f.write(digest)
    return KERNEL_LIB


def build_host(force: bool = False, verbose: bool = True) -> str:
    srcs = _sources("cpp")
    if not srcs:
        return ""
    os.makedirs(OUT_DIR, exist_ok=True)
    flags = ["-O3", "-std=c++17", "-fPIC", "-shared", "-fopenmp"]
    digest = _digest(srcs, " ".join(flags))
    if not force and _stamp_ok(HOST_LIB, digest):
        return HOST_LIB
    tmp = HOST_LIB + ".tmp"
    _run([CXX, *flags, "-I", os.path.join(HERE, "host"), *srcs, "-o", tmp])
    os.replace(tmp, HOST_LIB)
    with open(HOST_LIB + ".sha256", "w") as f:
        f.write(digest)
    if verbose:
        print(f"[build] host runtime -> {os.path.relpath(HOST_LIB, PKG)}", flush=True)
    return HOST_LIB


def build_host_sanitized(out_path: str, sanitizers: str = "address,undefined") -> str:
    """Debug target: the host runtime sources linked with the edge-case driver
    ``host/check/sanitize_dataio.cpp`` into one executable under ASan + UBSan.  GPU ASan is not
    available for gfx950 here, so the sanitized target is the host code only.  Not part of
    :func:`build_all`; ``tests/test_host_sanitize.py`` builds and runs it."""
    srcs = _sources("cpp") + [os.path.join(HERE, "host", "check", "sanitize_dataio.cpp")]
    flags = ["-O1", "-g", "-std=c++17", "-fopenmp", f"-fsanitize={sanitizers}",
             "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"]
    _run([CXX, *flags, "-I", os.path.join(HERE, "host"), *srcs, "-o", out_path])
    return out_path


def build_all(force: bool = False, jobs: int = 4, verbose: bool = True):
    return build_kernels(force, jobs, verbose), build_host(force, verbose)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    a = ap.parse_args(argv)
    k, h = build_all(a.force, a.jobs)
    print(k)
    if h:
        print(h)


if __name__ == "__main__":
    sys.exit(main())
