#!/usr/bin/env python3
"""Build the kernel library with extra preprocessor flags into _native/variants/<name>/ for A/B
runs: ``python tools/build_variant.py chains1 -DBWD_CHAINS=1`` then on the GPU
``DINUNET_KERNEL_LIB=dinunet_implementations_amd/_native/variants/chains1/libdinunet_kernels.so``.
"""
import concurrent.futures as cf
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dinunet_implementations_amd.csrc import build as B  # noqa: E402


def main():
    name, flags = sys.argv[1], sys.argv[2:]
    out = os.path.join(B.OUT_DIR, "variants", name)
    os.makedirs(out, exist_ok=True)
    objs = []

    def one(src):
        obj = os.path.join(out, os.path.basename(src) + ".o")
        B._run([B.HIPCC, *B.HIP_FLAGS, *B.FILE_FLAGS.get(os.path.basename(src), []), *flags,
                "-I", os.path.join(B.HERE, "kernels"), "-c", src, "-o", obj])
        return obj
    with cf.ThreadPoolExecutor(4) as ex:
        objs = list(ex.map(one, B._sources("hip")))
    lib = os.path.join(out, "libdinunet_kernels.so")
    B._run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", *objs, "-o", lib])
    for o in objs:
        os.remove(o)
    print(lib)


if __name__ == "__main__":
    main()
