"""MNIST IDX files and the PNG tree DLI ingests (replaces ``convert_mnist.py``).

* ``read(dataset, path)`` keeps the reference API and return value
  ``(labels, pixels, size, rows, cols)`` (``convert_mnist.py:15-35``): big-endian
  headers ``>II`` (labels) / ``>IIII`` (images).  ``.gz`` files are accepted.
* ``write_dataset(labels, data, size, rows, cols, output_dir)`` writes
  ``output_dir/{0..9}/{index}.png`` 28×28 grayscale (``convert_mnist.py:37-57``)
  with a zlib-based PNG encoder (pypng is not installed here).
* ``load_png_tree(dir)`` reads such a tree back (label = sub-folder name).
"""
from __future__ import annotations

import gzip
import os
import struct
import zlib
from typing import Iterable, List, Optional, Tuple

import numpy as np

FILES = {
    "training": ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
    "testing": ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte"),
}
ALIASES = {"train": "training", "test": "testing", "t10k": "testing"}


def _open(path: str):
    for cand in (path, path + ".gz", path.replace("-idx", ".idx")):
        if os.path.exists(cand):
            return gzip.open(cand, "rb") if cand.endswith(".gz") else open(cand, "rb")
    raise FileNotFoundError(path)


def read_idx_labels(path: str) -> np.ndarray:
    with _open(path) as f:
        magic, n = struct.unpack(">II", f.read(8))
        if magic != 2049:
            raise ValueError(f"{path}: bad IDX label magic {magic}")
        return np.frombuffer(f.read(n), dtype=np.uint8).astype(np.int32)


def read_idx_images(path: str) -> np.ndarray:
    with _open(path) as f:
        magic, n, rows, cols = struct.unpack(">IIII", f.read(16))
        if magic != 2051:
            raise ValueError(f"{path}: bad IDX image magic {magic}")
        return np.frombuffer(f.read(n * rows * cols), dtype=np.uint8).reshape(n, rows, cols)


def read(dataset: str = "training", path: str = "."):
    """Reference-compatible reader: returns (labels, pixels, size, rows, cols)."""
    dataset = ALIASES.get(dataset, dataset)
    if dataset not in FILES:
        raise ValueError("dataset must be 'testing' or 'training'")
    fi, fl = FILES[dataset]
    labels = read_idx_labels(os.path.join(path, fl))
    imgs = read_idx_images(os.path.join(path, fi))
    n, rows, cols = imgs.shape
    return labels, imgs.reshape(-1), n, rows, cols


def write_idx(path: str, images: np.ndarray, labels: np.ndarray) -> Tuple[str, str]:
    """Write an IDX pair (used to build test fixtures and synthetic exports)."""
    n, rows, cols = images.shape
    ipath, lpath = path + "-images-idx3-ubyte", path + "-labels-idx1-ubyte"
    with open(ipath, "wb") as f:
        f.write(struct.pack(">IIII", 2051, n, rows, cols))
        f.write(np.ascontiguousarray(images, dtype=np.uint8).tobytes())
    with open(lpath, "wb") as f:
        f.write(struct.pack(">II", 2049, n))
        f.write(np.asarray(labels, dtype=np.uint8).tobytes())
    return ipath, lpath


# ------------------------------------------------------------------ PNG
def png_encode_gray(img: np.ndarray) -> bytes:
    """8-bit grayscale, non-interlaced PNG (filter type 0 per row)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape

    def chunk(t: bytes, data: bytes) -> bytes:
        return struct.pack(">I", len(data)) + t + data + struct.pack(">I", zlib.crc32(t + data) & 0xFFFFFFFF)

    raw = b"".join(b"\x00" + img[r].tobytes() for r in range(h))
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 0, 0, 0, 0)) +
            chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))


def write_dataset(labels, data, size: int, rows: int, cols: int, output_dir: str, verbose: bool = False) -> None:
    """Reference-compatible PNG tree writer (convert_mnist.py:37-57)."""
    data = np.asarray(data, dtype=np.uint8).reshape(size, rows, cols)
    for i in range(10):
        os.makedirs(os.path.join(output_dir, str(i)), exist_ok=True)
    for i, label in enumerate(np.asarray(labels).reshape(-1)):
        out = os.path.join(output_dir, str(int(label)), f"{i}.png")
        if verbose:
            print("writing " + out)
        with open(out, "wb") as h:
            h.write(png_encode_gray(data[i]))


def decode_image(path: str, channels: int = 1, size: int = 28) -> np.ndarray:
    """Decode PNG/JPEG to uint8 [size, size, channels] with centre crop/pad
    (``tf.image.resize_image_with_crop_or_pad``, inference.py:73)."""
    from PIL import Image
    with Image.open(path) as im:
        im = im.convert("L" if channels == 1 else "RGB")
        a = np.asarray(im, dtype=np.uint8)
    if a.ndim == 2:
        a = a[..., None]
    return crop_or_pad(a, size, size)


def crop_or_pad(a: np.ndarray, th: int, tw: int) -> np.ndarray:
    h, w, c = a.shape
    out = np.zeros((th, tw, c), dtype=a.dtype)
    # TF semantics: crop centred, pad centred (offset = diff // 2)
    sy, sx = max((h - th) // 2, 0), max((w - tw) // 2, 0)
    dy, dx = max((th - h) // 2, 0), max((tw - w) // 2, 0)
    ch, cw = min(h, th), min(w, tw)
    out[dy:dy + ch, dx:dx + cw] = a[sy:sy + ch, sx:sx + cw]
    return out


def list_images(input_dir: str) -> List[str]:
    """``glob(input_dir/*.*)`` filtered to .jpg/.jpeg/.png (inference.py:38-42)."""
    d = os.path.expanduser(input_dir)
    names = sorted(os.listdir(d)) if os.path.isdir(d) else []
    return [os.path.join(d, n) for n in names if n.lower().endswith((".jpg", ".jpeg", ".png"))]


def load_png_tree(root: str, channels: int = 1, limit: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
    imgs, labels = [], []
    for lab in sorted(os.listdir(root)):
        sub = os.path.join(root, lab)
        if not (os.path.isdir(sub) and lab.isdigit()):
            continue
        for p in list_images(sub):
            imgs.append(decode_image(p, channels).reshape(-1))
            labels.append(int(lab))
            if limit and len(imgs) >= limit:
                break
    if not imgs:
        raise ValueError(f"no images under {root}")
    return np.stack(imgs), np.asarray(labels, dtype=np.int32)
