"""GPU-resident dataset + on-device shuffle/gather.

Replaces the reference's queue-runner pipeline (``string_input_producer`` →
``TFRecordReader`` → ``shuffle_batch(num_threads=2, capacity=1000+3B,
min_after_dequeue=1000)``, ``mnist_input.py:58-71``).  MNIST is 47 MB as uint8,
so the whole split lives in HBM; each step is ONE gather+normalise kernel
(``prep_images``: ``x/255 - 0.5``, optional 1→3 channel replication) writing
straight into the executor's input buffer.  Shuffling is a full-epoch
permutation (stronger than the reference's 1000-example shuffle buffer),
computed per batch as a keyed Feistel bijection of the stream position
(``perm_positions``: no sort, no per-epoch state; the data order is a pure
function of (seed, position), so ``seek(step)`` resumes it exactly).

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
        if out_images.dtype == torch.float32:     # --precision fp32 input buffer
            kernels().f32_prep_images(ds.images, idx, ds.labels, out_images, out_labels, ds.hw, ds.channels, cdst)
        else:
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
        self._bf16: Optional[torch.Tensor] = None

    def bf16_images(self) -> torch.Tensor:
        """The whole split normalised once (x/255 - 0.5, bf16, [n, hw*channels]): the
        resident input of the bf16 dataset-gather mode (HipNet.bind_u8_input).  Built
        with the same K10 kernel as the per-step gather, so it is bitwise what
        ``prep_images`` would write for every row."""
        if self._bf16 is None:
            n = len(self)
            out = torch.empty(n, self.hw * self.channels, dtype=torch.bfloat16, device=self.device)
            labs = torch.empty(n, dtype=torch.int32, device=self.device)
            gather_into(self, torch.arange(n, device=self.device), out.view(n, self.hw, self.channels), labs)
            self._bf16 = out
        return self._bf16

    def __len__(self) -> int:
        return int(self.images.shape[0])


M32 = 0xFFFFFFFF


def _mix32(x):
    """32-bit integer hash (works on Python ints and int64 tensors; wraps like uint32)."""
    x = ((x ^ (x >> 16)) * 0x7feb352d) & M32
    x = ((x ^ (x >> 15)) * 0x846ca68b) & M32
    return x ^ (x >> 16)


def _half_bits(n: int) -> int:
    h = 1
    while (1 << (2 * h)) < n:
        h += 1
    return h


def perm_positions(start: int, n: int, N: int, seed: int, device=None, out: Optional[torch.Tensor] = None,
                   labels: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
    """Dataset rows of stream positions start..start+n-1: position p -> F_e(p mod N),
    e = p // N, F_e a 4-round keyed Feistel bijection on [0, 4^h) restricted to
    [0, N) by cycle walking.  Every epoch is a full permutation of the dataset.
    On a GPU this is the ``perm_positions`` HIP kernel (misc.hip), bit-identical.
    ``labels`` = (dataset labels, out labels): also gather the rows' labels (one
    launch on the GPU)."""
    h = _half_bits(N)
    seed &= M32
    dev = torch.device(device) if device is not None else (out.device if out is not None else torch.device("cpu"))
    if dev.type == "cuda":
        if out is None:
            out = torch.empty(n, dtype=torch.int64, device=dev)
        if labels is not None:
            kernels().perm_positions(out[:n], int(start), int(N), int(seed), int(h), labels[0], labels[1][:n])
        else:
            kernels().perm_positions(out[:n], int(start), int(N), int(seed), int(h))
        return out[:n]
    mask = (1 << h) - 1
    p = torch.arange(start, start + n, dtype=torch.int64)
    e = p // N
    x = p - e * N
    ek = _mix32((e & M32) ^ 0x9E3779B9) ^ seed
    keys = [_mix32((ek + 0x85EBCA77 * (r + 1)) & M32) for r in range(4)]

    def F(v):
        L, R = v >> h, v & mask
        for r in range(4):
            L, R = R, L ^ (_mix32(R ^ keys[r]) & mask)
        return (L << h) | R

    x = F(x)
    while True:
        bad = x >= N
        if not bool(bad.any()):
            break
        x = torch.where(bad, F(x), x)
    if labels is not None:
        labels[1][:n].copy_(labels[0].to(x.device)[x])
    if out is not None:
        out[:n].copy_(x)
        return out[:n]
    return x


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
        self.cdst = int(out_images.shape[-1])
        # sharded ranks walk ONE global order (same key); unsharded ones each their own
        self.seed = (seed if shard else seed + 7919 * rank) & M32
        self.idx = torch.empty(self.B, dtype=torch.int64, device=ds.device)
        self.pos = 0          # stream position of the next global batch
        self._ahead = None    # position whose rows + labels an optimizer launch already wrote

    @property
    def epoch(self) -> int:
        return self.pos // len(self.ds)

    def seek(self, step: int) -> None:
        """Position the stream at global step ``step`` (resume from a checkpoint)."""
        self.pos = int(step) * self.global_batch

    def lookahead_job(self) -> Optional[tuple]:
        """The NEXT local batch's ``perm_positions`` job -- (rows out, dataset labels, labels out,
        start, N, seed, h) -- for the current step's optimizer launch to run in extra blocks
        (``HipNet.next_input_job``, misc.hip ``PermJob``); the next ``next()`` then launches
        nothing.  Only for the resident-dataset shuffle (``idx_out``) with full batches, and
        only where nothing else writes the index / label buffers between the optimizer and
        the next ``next()`` (bench.py; not the CLI loop, which evaluates into them)."""
        if not (self.shuffle and self.idx_out is not None and self.idx_out.is_cuda and self.ds.device.type == "cuda"):
            return None
        N = len(self.ds)
        start = self.pos + (self.rank * self.B if self.shard else 0)
        self._ahead = self.pos
        return (self.idx_out[:self.B], self.ds.labels, self.out_labels[:self.B], int(start), int(N), int(self.seed),
                _half_bits(N))

    def next(self, nb: Optional[int] = None) -> int:
        """Gather the next local batch into the output buffers; returns its size."""
        nb = self.B if nb is None else nb
        ahead, self._ahead = self._ahead, None
        if ahead is not None and ahead == self.pos and nb == self.B:
            self.pos += self.global_batch   # the previous optimizer launch wrote this batch
            return nb
        start = self.pos + (self.rank * self.B if self.shard else 0)
        N = len(self.ds)
        if (self.shuffle and self.idx_out is None and self.ds.device.type == "cuda" and self.ds.hw == 784
                and self.ds.channels == 1 and self.cdst == 1 and self.out_images.dtype == torch.bfloat16):
            # one kernel: Feistel row + gather + normalise (+ labels)
            kernels().prep_images_perm(self.ds.images, self.ds.labels, self.out_images, self.out_labels, nb,
                                       int(start), int(self.seed), _half_bits(N))
            self.pos += self.global_batch
            return nb
        if self.shuffle and self.idx_out is not None and self.idx_out.is_cuda:
            # resident-dataset input: the Feistel rows straight into the executor's index
            # buffer, labels gathered in the same launch
            perm_positions(start, nb, N, self.seed, out=self.idx_out, labels=(self.ds.labels, self.out_labels))
            self.pos += self.global_batch
            return nb
        if self.shuffle:
            idx = perm_positions(start, nb, N, self.seed, out=self.idx)
        else:
            idx = torch.remainder(torch.arange(start, start + nb, device=self.ds.device), N)
        if self.idx_out is not None:
            self.idx_out[:nb].copy_(idx)
            torch.index_select(self.ds.labels, 0, idx, out=self.out_labels[:nb])
        else:
            gather_into(self.ds, idx, self.out_images, self.out_labels)
        self.pos += self.global_batch
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
