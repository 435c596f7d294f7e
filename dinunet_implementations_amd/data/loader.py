"""HBM-resident batch loader.

The reference iterates a torch ``DataLoader`` whose workers parse files and collate float64
batches that are then copied host->device every step (``comps/fs/__init__.py:51``).  Here the
split already sits in device memory as one ``[N, ...]`` tensor; an epoch is a device-side
permutation and every batch is a single gather (or a contiguous slice when not shuffling).
``drop_last`` follows ``dataloader_args`` (the reference sets it for train: ``local.py:29``,
BatchNorm cannot take a 1-sample batch).
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import torch


class DeviceLoader:
    def __init__(self, inputs: torch.Tensor, labels: torch.Tensor, batch_size: int,
                 shuffle: bool = False, drop_last: bool = False, seed: int = 0,
                 index: Optional[torch.Tensor] = None, merge_singleton: bool = True):
        self.inputs = inputs
        self.labels = labels
        self.index = index  # global sample ids (for logging predictions), same order as inputs
        self.batch_size = max(1, int(batch_size))
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.epoch = 0
        self.seed = seed
        # a trailing 1-sample batch breaks batch-statistics BatchNorm (the FS model normalises
        # with batch stats even in eval): fold it into the previous batch instead
        self.merge_singleton = merge_singleton
        self._gen = torch.Generator(device="cpu")
        self._pos = 0  # batches yielded by the current pass (resume position)

    def __len__(self):
        n = self.inputs.shape[0]
        if self.drop_last:
            return n // self.batch_size
        nb = (n + self.batch_size - 1) // self.batch_size
        if self.merge_singleton and nb > 1 and n % self.batch_size == 1:
            nb -= 1
        return nb

    @property
    def num_samples(self) -> int:
        return int(self.inputs.shape[0])

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def _spans(self) -> Iterator[Tuple[int, int, Optional[torch.Tensor]]]:
        """One pass: ``(start, end, perm)`` per batch (``perm`` None when not shuffling)."""
        n = self.inputs.shape[0]
        dev = self.inputs.device
        if self.shuffle:
            self._gen.manual_seed(self.seed * 100003 + self.epoch)
            perm = torch.randperm(n, generator=self._gen).to(dev, non_blocking=True)
        else:
            perm = None
        self.epoch += 1
        self._pos = 0
        nb = len(self)
        for b in range(nb):
            self._pos = b + 1
            s = b * self.batch_size
            e = n if b == nb - 1 and not self.drop_last else min(n, s + self.batch_size)
            yield s, e, perm

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
        dev = self.inputs.device
        for s, e, perm in self._spans():
            if perm is None:
                ix = torch.arange(s, e, device=dev)
                yield self.inputs[s:e], self.labels[s:e], ix
            else:
                ix = perm[s:e]
                yield self.inputs.index_select(0, ix), self.labels.index_select(0, ix), ix

    def iter_indices(self) -> Iterator[torch.Tensor]:
        """The sample indices of the batches :meth:`__iter__` would yield, same passes, same
        shuffles, same resume position, without gathering the batches (a device-fed epoch
        gathers them on the device: ``runtime.feed.DeviceFeed``)."""
        dev = self.inputs.device
        for s, e, perm in self._spans():
            yield torch.arange(s, e, device=dev) if perm is None else perm[s:e]

    @property
    def full_batches(self) -> bool:
        """Every batch of a pass holds exactly ``batch_size`` samples."""
        n = self.inputs.shape[0]
        return n >= self.batch_size and (self.drop_last or n % self.batch_size == 0)

    # ---- resume ------------------------------------------------------------------------------
    def state(self) -> dict:
        """Position for an exact resume: passes started and batches consumed in the current one
        (the shuffle of a pass is a pure function of ``seed`` and its pass number)."""
        return {"epoch": int(self.epoch), "pos": int(self._pos)}

    def resume_iter(self, state: dict, indices: bool = False):
        """An iterator that continues where :meth:`state` was taken (of batch indices only,
        :meth:`iter_indices`, with ``indices``)."""
        self.epoch = max(0, int(state.get("epoch", 0)) - 1)
        it = self.iter_indices() if indices else iter(self)
        for _ in range(int(state.get("pos", 0))):
            next(it, None)
        return it
