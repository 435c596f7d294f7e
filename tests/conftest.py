import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built kernels")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


REF_DATA = "/root/reference/datasets/test_fsl"


@pytest.fixture
def fs_data_root():
    """The reference's shipped 5-site FreeSurfer simulator data (read-only), or a synthetic copy."""
    if os.path.isdir(REF_DATA):
        return REF_DATA
    from dinunet_implementations_amd.data.synthetic import make_fs_sites
    import tempfile
    d = tempfile.mkdtemp()
    return make_fs_sites(d, sites=5, subjects=(40, 30, 50, 40, 60))
