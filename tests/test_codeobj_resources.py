"""Resource audit of the built gfx950 code objects (CPU only: reads the ELF notes of the objects
``csrc/build.py`` compiled).

Scratch (private segment) use in a hot kernel means registers went to memory: the head's layer-0
kernel once indexed a register array from a non-unrolled loop and every element made an
HBM-latency round trip (14 us of a 20 us kernel).  Kernels that run every training step must
keep ``private_segment_fixed_size == 0``; the few instantiations for configurations the
benchmark does not take (wide-batch LSTM backward) are listed with their known spill counts.
"""
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "dinunet_implementations_amd", "_native", "obj")
LLVM = "/opt/rocm/lib/llvm/bin"

# (kernel-name regex) -> max tolerated private segment bytes
ALLOWED = {
    # BR = 16 backward with a per-step output gradient (sequence-output mode, batch > 512 only;
    # the ICA model's temporal-mean mode does not spill)
    r"lstm_bwd_kernelILi192ELi16ELb1E": 96,
    # rank-dAD's one-launch power iteration at rank bound 16 with MIXED per-layer ranks (some
    # layer above 12; one rank for all layers takes the spill-free exact-rank kernels, the
    # compspec default rank 10 among them)
    r"lr_persist_kernelILi16ELb0E": 192,
}


def _tool(name):
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else shutil.which(name)


def _kernel_notes():
    objcopy, bundler, readelf = (_tool("llvm-objcopy"), _tool("clang-offload-bundler"),
                                 _tool("llvm-readelf"))
    if not (objcopy and bundler and readelf) or not glob.glob(os.path.join(OBJ, "*.o")):
        pytest.skip("ROCm LLVM tools or built objects missing")
    out = {}
    for obj in sorted(glob.glob(os.path.join(OBJ, "*.hip.o"))):
        tmp = obj + ".fatbin.tmp"
        co = obj + ".gfx950.tmp"
        try:
            subprocess.run([objcopy, f"--dump-section=.hip_fatbin={tmp}", obj], check=True,
                           capture_output=True)
            subprocess.run([bundler, "--unbundle", "--type=o", f"--input={tmp}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                           check=True, capture_output=True)
            notes = subprocess.run([readelf, "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
        finally:
            for f in (tmp, co):
                if os.path.exists(f):
                    os.remove(f)
        name = None
        for line in notes.splitlines():
            m = re.match(r"\s+\.name:\s+(\S+)", line)
            if m:
                name = m.group(1)
            m = re.match(r"\s+\.private_segment_fixed_size:\s+(\d+)", line)
            if m and name:
                out[name] = int(m.group(1))
    return out


def test_no_scratch_in_step_kernels():
    notes = _kernel_notes()
    assert any("gemm_kernel" in k for k in notes), "gemm kernels not found in the objects"
    bad = {}
    for name, scratch in notes.items():
        limit = next((v for pat, v in ALLOWED.items() if re.search(pat, name)), 0)
        if scratch > limit:
            bad[name] = scratch
    assert not bad, f"kernels using scratch (register spills / dynamic indexing): {bad}"
