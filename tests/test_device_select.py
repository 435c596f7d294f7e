"""Per-site device selection from the site input's ``gpus`` (reference
``datasets/icalstm/inputspec.json:6-10``: site r -> [r]; ``datasets/test_fsl/inputspec.json:15-17``:
[] = CPU-only), checked without a GPU."""
import pytest
import torch

from dinunet_implementations_amd.parallel.group import resolve_device


def test_gpus_missing_is_this_ranks_gpu():
    assert resolve_device(None, local_rank=3, n_devices=8) == torch.device("cuda", 3)
    assert resolve_device(None, local_rank=9, n_devices=8) == torch.device("cuda", 1)
    assert resolve_device(None, local_rank=0, n_devices=0) == torch.device("cpu")


def test_gpus_empty_means_cpu():
    assert resolve_device([], local_rank=2, n_devices=8) == torch.device("cpu")


def test_gpus_list_picks_the_first_id():
    assert resolve_device([1], local_rank=0, n_devices=8) == torch.device("cuda", 1)
    with pytest.warns(RuntimeWarning, match="not used"):  # extra ids are reported, not dropped
        assert resolve_device([2, 3], local_rank=0, n_devices=8) == torch.device("cuda", 2)
    assert resolve_device(5, local_rank=0, n_devices=8) == torch.device("cuda", 5)


def test_gpus_out_of_range():
    with pytest.raises(ValueError, match="does not exist"):
        resolve_device([8], local_rank=8, world=9, backend="nccl", n_devices=8)
    with pytest.warns(RuntimeWarning):  # sites rehearsed on fewer GPUs wrap around
        assert resolve_device([9], local_rank=0, n_devices=8) == torch.device("cuda", 1)


def test_rccl_site_must_own_gpu_local_rank():
    # one process per GPU over RCCL: site r lists GPU r (reference ICA inputspec)
    assert resolve_device([1], local_rank=1, world=2, backend="nccl", n_devices=2) == torch.device("cuda", 1)
    with pytest.raises(ValueError, match="LOCAL_RANK"):
        resolve_device([0], local_rank=1, world=2, backend="nccl", n_devices=2)
    # gloo rehearsal of several sites on one GPU: any id is fine
    assert resolve_device([0], local_rank=1, world=2, backend="gloo", n_devices=1) == torch.device("cuda", 0)


def test_gpus_without_visible_gpu_falls_back_to_cpu():
    with pytest.warns(RuntimeWarning):
        assert resolve_device([0], local_rank=0, n_devices=0) == torch.device("cpu")


def test_site_runner_and_local_node_resolve_from_config():
    from dinunet_implementations_amd.compat.nodes import LocalNode
    node = LocalNode()
    assert node.device == torch.device("cpu")  # resolved from the input at setup


def test_ranks_beyond_the_inputspec_take_their_own_gpu():
    """run.py gives rank r the input specs[r % n]: the reference icalstm spec pins site 0 to GPU 0
    and site 1 to GPU 1, so under RCCL with 4 ranks ranks 2 and 3 must NOT inherit those pins
    (they would conflict with LOCAL_RANK and raise): they take GPU LOCAL_RANK."""
    from dinunet_implementations_amd.run import site_gpus
    specs = [{"gpus": [0]}, {"gpus": [1]}]
    devs = []
    for rank in range(4):
        g = site_gpus(specs[rank % 2], rank, len(specs))
        devs.append(resolve_device(g, local_rank=rank, world=4, backend="nccl", n_devices=8))
    assert devs == [torch.device("cuda", r) for r in range(4)]
    # the spec's own ranks keep their pin, CPU-only sites keep the CPU
    assert site_gpus({"gpus": [1]}, 1, 2) == [1]
    assert site_gpus({"gpus": []}, 0, 2) == []
    assert resolve_device(site_gpus({"gpus": []}, 0, 2), n_devices=8) == torch.device("cpu")
