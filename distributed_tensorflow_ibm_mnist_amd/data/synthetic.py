"""Synthetic MNIST-shaped data (no network in this environment: SURVEY.md §4).

``synthetic://N[?seed=S&noise=F&style=glyph|hand]`` yields N 28×28 uint8 images
with labels 0-9.  Each class has a fixed random "stroke" template (a smooth path
of 6 control points, like a pen-drawn glyph).

* ``glyph`` (default): every sample is its class template shifted by up to
  ±2 px, intensity-jittered, with additive noise -- fast, and easy.
* ``hand``: every sample re-draws its class path from control points jittered
  per sample (σ 1.6 px), rotated (±15°), scaled (0.85-1.15), with a random pen
  width and shift -- intra-class variability like handwriting, so
  steps-to-99%-train-accuracy (BASELINE.json) measures real learning.

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


def _control_points(seed: int = 0, classes: int = 10) -> torch.Tensor:
    g = torch.Generator().manual_seed(1000 + seed)
    return torch.stack([4 + torch.rand(6, 2, generator=g) * 20 for _ in range(classes)])  # [10, 6, 2]


def _hand(labels: torch.Tensor, g: torch.Generator, dev: torch.device, chunk: int = 1024) -> torch.Tensor:
    n = labels.numel()
    cp = _control_points().to(dev)[labels]                                       # [n, 6, 2]
    cp = cp + 1.6 * torch.randn(cp.shape, generator=g, device=dev)
    ang = (torch.rand(n, generator=g, device=dev) - 0.5) * (torch.pi / 6)
    sc = 0.85 + 0.3 * torch.rand(n, generator=g, device=dev)
    c, s_ = torch.cos(ang) * sc, torch.sin(ang) * sc
    ctr = cp - 14.0
    cp = torch.stack([c[:, None] * ctr[..., 0] - s_[:, None] * ctr[..., 1],
                      s_[:, None] * ctr[..., 0] + c[:, None] * ctr[..., 1]], -1) + 14.0
    cp = cp + (torch.rand(n, 1, 2, generator=g, device=dev) - 0.5) * 4.0        # shift ±2 px
    width = 0.9 + 0.9 * torch.rand(n, generator=g, device=dev)
    t = torch.linspace(0, 1, 12, device=dev)
    path = (cp[:, :-1, None] * (1 - t[None, None, :, None]) + cp[:, 1:, None] * t[None, None, :, None])
    path = path.reshape(n, -1, 2)                                                # [n, 60, 2]
    ar = torch.arange(28, dtype=torch.float32, device=dev)
    out = torch.empty(n, 28, 28, device=dev)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        py, px = path[a:b, :, 0], path[a:b, :, 1]
        d2 = (ar[None, None, :, None] - py[:, :, None, None]) ** 2 + (ar[None, None, None, :] - px[:, :, None, None]) ** 2
        img = torch.exp(-d2.amin(1) / (2 * width[a:b, None, None] ** 2))
        out[a:b] = img / img.amax((1, 2), keepdim=True).clamp_min(1e-6)
    return out


def make_synthetic(n: int, seed: int = 0, channels: int = 1, noise: float = 0.25,
                   device: str | torch.device = "cpu", style: str = "glyph") -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (images uint8 [n, 28*28*channels] HWC-flattened, labels int32 [n])."""
    dev = torch.device(device)
    if style == "hand":
        g = torch.Generator(device=dev).manual_seed(seed)
        labels = torch.randint(0, 10, (n,), generator=g, device=dev)
        imgs = _hand(labels, g, dev)
        scale = 0.6 + 0.4 * torch.rand(n, 1, 1, generator=g, device=dev)
        imgs = imgs * scale + noise * torch.rand(n, 28, 28, generator=g, device=dev)
        u8 = (imgs.clamp(0, 1) * 255).round().to(torch.uint8)
        if channels > 1:
            u8 = u8[..., None].expand(n, 28, 28, channels)
        return u8.reshape(n, -1).contiguous(), labels.to(torch.int32)
    if style != "glyph":
        raise ValueError(f"unknown synthetic style {style!r}")
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
    if "style" in q:
        opts["style"] = q["style"]
    return n, opts


def as_numpy(images: torch.Tensor, labels: torch.Tensor) -> Tuple[np.ndarray, np.ndarray]:
    return images.cpu().numpy(), labels.cpu().numpy()
