"""Synthetic MNIST-shaped data (no network in this environment: SURVEY.md §4).

``synthetic://N[?seed=S&noise=F]`` yields N 28×28 uint8 images with labels 0-9.
Each class has a fixed random "stroke" template (a smooth blob path, like a
pen-drawn glyph); every sample is its class template shifted by up to ±2 px,
intensity-jittered, with additive noise.  The task is learnable (so
steps-to-99%-train-accuracy is meaningful) but not trivially separable at init.

Generation is vectorised torch (CPU or GPU) and deterministic in the seed.
"""
from __future__ import annotations

import urllib.parse
from typing import Tuple

import numpy as np
import torch


def _templates(seed: int, classes: int = 10, size: int = 28) -> torch.Tensor:
    g = torch.Generator().manual_seed(1000 + seed)
    yy, xx = torch.meshgrid(torch.arange(size, dtype=torch.float32), torch.arange(size, dtype=torch.float32),
                            indexing="ij")
    out = torch.zeros(classes, size, size)
    for c in range(classes):
        # a random smooth path of 6 control points inside the 20x20 centre box
        pts = 4 + torch.rand(6, 2, generator=g) * 20
        t = torch.linspace(0, 1, 40)
        path = []
        for i in range(5):
            a, b = pts[i], pts[i + 1]
            path.append(a[None] * (1 - t[:, None]) + b[None] * t[:, None])
        path = torch.cat(path)  # [200, 2]
        d2 = (yy[None] - path[:, 0, None, None]) ** 2 + (xx[None] - path[:, 1, None, None]) ** 2
        img = torch.exp(-d2 / (2 * 1.3 ** 2)).amax(0)
        out[c] = img / img.max()
    return out


def make_synthetic(n: int, seed: int = 0, channels: int = 1, noise: float = 0.25,
                   device: str | torch.device = "cpu") -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (images uint8 [n, 28*28*channels] HWC-flattened, labels int32 [n])."""
    dev = torch.device(device)
    tmpl = _templates(0).to(dev)  # class templates are shared by every split (train/test/val)
    g = torch.Generator(device=dev).manual_seed(seed)
    labels = torch.randint(0, 10, (n,), generator=g, device=dev)
    imgs = tmpl[labels]  # [n, 28, 28]
    # random integer shifts in [-2, 2] (per sample) via roll on a padded canvas
    pad = 2
    canvas = torch.nn.functional.pad(imgs, (pad, pad, pad, pad))
    sy = torch.randint(0, 2 * pad + 1, (n,), generator=g, device=dev)
    sx = torch.randint(0, 2 * pad + 1, (n,), generator=g, device=dev)
    ar = torch.arange(28, device=dev)
    rows = (sy[:, None] + ar[None]).clamp_(0, 28 + 2 * pad - 1)
    cols = (sx[:, None] + ar[None]).clamp_(0, 28 + 2 * pad - 1)
    imgs = canvas[torch.arange(n, device=dev)[:, None, None], rows[:, :, None], cols[:, None, :]]
    scale = 0.6 + 0.4 * torch.rand(n, 1, 1, generator=g, device=dev)
    imgs = imgs * scale + noise * torch.rand(n, 28, 28, generator=g, device=dev)
    u8 = (imgs.clamp(0, 1) * 255).round().to(torch.uint8)
    if channels > 1:
        u8 = u8[..., None].expand(n, 28, 28, channels)
    return u8.reshape(n, -1).contiguous(), labels.to(torch.int32)


def parse_uri(uri: str) -> Tuple[int, dict]:
    """``synthetic://60000?seed=1&noise=0.3`` -> (60000, {'seed': 1, 'noise': 0.3})."""
    u = urllib.parse.urlparse(uri)
    n = int(u.netloc or u.path.strip("/") or 60000)
    q = {k: v[-1] for k, v in urllib.parse.parse_qs(u.query).items()}
    opts = {}
    if "seed" in q:
        opts["seed"] = int(q["seed"])
    if "noise" in q:
        opts["noise"] = float(q["noise"])
    return n, opts


def as_numpy(images: torch.Tensor, labels: torch.Tensor) -> Tuple[np.ndarray, np.ndarray]:
    return images.cpu().numpy(), labels.cpu().numpy()
