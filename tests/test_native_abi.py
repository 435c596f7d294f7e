"""The ctypes signatures registered in ``ops`` match the C ABI declared in csrc/kernels/*.hip.

A wrong argument count only shows up on a GPU box otherwise (``TypeError`` at call time, or
worse, a shifted argument): this parses every ``DN_API`` declaration and compares arities.
"""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, "dinunet_implementations_amd", "csrc", "kernels")


def _c_signatures():
    sigs = {}
    for path in glob.glob(os.path.join(KDIR, "*.hip")):
        src = open(path).read()
        for m in re.finditer(r"DN_API\s+[\w\s\*]+?\b(dn_\w+)\s*\(([^)]*)\)", src):
            args = m.group(2).strip()
            sigs[m.group(1)] = 0 if args in ("", "void") else len(args.split(","))
    return sigs


def test_registered_arities_match_c_declarations():
    import dinunet_implementations_amd.ops  # noqa: F401  (registers every signature)
    from dinunet_implementations_amd.ops import _lib
    csigs = _c_signatures()
    assert "dn_gemm" in csigs and "dn_head_fwd" in csigs
    bad = {}
    for name, argtypes in _lib._SIGS.items():
        if name not in csigs:
            bad[name] = "not declared in csrc/kernels"
        elif len(argtypes) != csigs[name]:
            bad[name] = f"ctypes {len(argtypes)} vs C {csigs[name]}"
    assert not bad, bad


def test_peer_exchange_argument_block_matches_library():
    """``parallel.peer._PxArgs`` (ctypes) and peer.hip's PxArgs must agree byte for byte: the
    launcher copies the block into the kernel arguments."""
    import ctypes
    from dinunet_implementations_amd.ops import _lib
    if not _lib.native_available():
        pytest.skip("kernel library not built")
    from dinunet_implementations_amd.parallel import peer
    assert ctypes.sizeof(peer._PxArgs) == int(_lib.lib().dn_peer_args_size())
    assert int(_lib.lib().dn_peer_handle_size()) == 64
