"""GPU-resident dataset + on-device shuffle/gather.

Replaces the reference's queue-runner pipeline (``string_input_producer`` →
``TFRecordReader`` → ``shuffle_batch(num_threads=2, capacity=1000+3B,
min_after_dequeue=1000)``, ``mnist_input.py:58-71``).  MNIST is 47 MB as uint8,
so the whole split lives in HBM; each step is ONE gather+normalise kernel
(``prep_images``: ``x/255 - 0.5``, optional 1→3 channel replication) writing
straight into the executor's input buffer.  Shuffling is a device-side
permutation per epoch (a full-epoch shuffle — stronger than the reference's
1000-example shuffle buffer).

Data parallel sharding: with ``shard=True`` every rank walks the
same global permutation and takes its slice of each global batch
(DistributedSampler semantics); ``shard=False`` reproduces the reference, where
every worker reads the whole file list in its own random order.
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import torch

from ..ops._ext import kernels


def gather_into(ds: "DeviceDataset", idx: torch.Tensor, out_images: torch.Tensor, out_labels: torch.Tensor) -> None:
    """K10 on the GPU; a torch equivalent on CPU (the gloo test path)."""
    cdst = int(out_images.shape[-1])
    if ds.device.type == "cuda":
        kernels().prep_images(ds.images, idx, ds.labels, out_images, out_labels, ds.hw, ds.channels, cdst)
        return
    nb = idx.numel()
    x = ds.images[idx].float().view(nb, ds.hw, ds.channels) * (1.0 / 255.0) - 0.5
    if ds.channels != cdst:
        x = x[..., :1].expand(nb, ds.hw, cdst)
    out_images.view(-1)[: nb * ds.hw * cdst].copy_(x.reshape(-1))
    out_labels[:nb].copy_(ds.labels[idx])


class DeviceDataset:
    def __init__(self, images: torch.Tensor, labels: torch.Tensor, device, hw: int = 784, channels: int = 1):
        assert images.dtype == torch.uint8 and images.dim() == 2
        assert images.shape[1] == hw * channels, (images.shape, hw, channels)
        self.device = torch.device(device)
        self.images = images.to(self.device).contiguous()
        self.labels = labels.to(self.device, torch.int32).contiguous()
        self.hw, self.channels = hw, channels

    def __len__(self) -> int:
        return int(self.images.shape[0])


class DeviceLoader:
    def __init__(self, ds: DeviceDataset, out_images: torch.Tensor, out_labels: torch.Tensor, rank: int = 0,
                 world: int = 1, seed: int = 0, shard: bool = True, shuffle: bool = True,
                 idx_out: Optional[torch.Tensor] = None):
        """``idx_out``: instead of gathering + normalising images into ``out_images``,
        write the batch's dataset indices there (the first fused conv reads the
        uint8 dataset itself: HipNet.bind_u8_input); labels are still gathered."""
        self.ds, self.out_images, self.out_labels = ds, out_images, out_labels
        self.idx_out = idx_out
        self.B = int(out_labels.shape[0])
        self.rank, self.world, self.shard, self.shuffle = rank, world, shard, shuffle
        self.global_batch = self.B * world if shard else self.B
        # One device permutation covers >= 16 global batches (several passes over
        # small datasets), so the sort behind randperm is amortised instead of
        # running every step when the global batch approaches the dataset size.
        self.reps = max(1, -(-16 * self.global_batch // len(ds))) if self.global_batch * 4 > len(ds) else 1
        self.cdst = int(out_images.shape[-1])
        self.gen = torch.Generator(device=ds.device)
        self.gen.manual_seed(seed if shard else seed + 7919 * rank)
        self.perm: Optional[torch.Tensor] = None
        self.cursor = 0
        self.epoch = 0
        self._new_epoch()

    def _new_epoch(self) -> None:
        n = len(self.ds) * self.reps
        if self.shuffle:
            self.perm = torch.randperm(n, generator=self.gen, device=self.ds.device) % len(self.ds)
        else:
            self.perm = torch.arange(n, device=self.ds.device) % len(self.ds)
        self.cursor = 0

    def next(self, nb: Optional[int] = None) -> int:
        """Gather the next local batch into the output buffers; returns its size."""
        nb = self.B if nb is None else nb
        if self.cursor + self.global_batch > self.perm.numel():
            self.epoch += 1
            self._new_epoch()
        start = self.cursor + (self.rank * self.B if self.shard else 0)
        idx = self.perm[start:start + nb]
        if self.idx_out is not None:
            self.idx_out[:nb].copy_(idx)
            torch.index_select(self.ds.labels, 0, idx, out=self.out_labels[:nb])
        else:
            gather_into(self.ds, idx, self.out_images, self.out_labels)
        self.cursor += self.global_batch
        return nb


def eval_batches(ds: DeviceDataset, out_images: torch.Tensor, out_labels: torch.Tensor) -> Iterator[int]:
    """Sequential pass over a split (no shuffle); yields the batch size of each step
    (the last one may be smaller: ``allow_smaller_final_batch``, inference.py:76-78)."""
    B = int(out_labels.shape[0])
    n = len(ds)
    ar = torch.arange(n, device=ds.device)
    for s in range(0, n, B):
        nb = min(B, n - s)
        gather_into(ds, ar[s:s + nb], out_images, out_labels)
        yield nb
