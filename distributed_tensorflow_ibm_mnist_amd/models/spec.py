"""Declarative model specs shared by the HIP executor and the PyTorch oracle.

A model is a sequential list of layer specs.  Tensor layouts follow the
reference (TF defaults): activations NHWC, conv weights ``[KH, KW, Cin, Cout]``,
dense weights ``[in, out]`` (``mnist_input.py:137-205``), so checkpoints keep
the reference's variable names *and* shapes.

Every weight carries the reference's init and weight-decay metadata:
``_variable_with_weight_decay(name, shape, stddev, wd)`` (``mnist_input.py:
90-115``) → ``w_std`` / ``wd``; biases ``tf.constant_initializer`` → ``b_init``.
"""
from __future__ import annotations

import dataclasses
import math
from typing import List, Optional, Tuple, Union


@dataclasses.dataclass
class Conv:
    name: str
    kh: int
    kw: int
    cin: int
    cout: int
    padding: str = "SAME"      # SAME | VALID, stride 1 (mnist_input.py:142,161)
    relu: bool = True
    w_std: float = 5e-2
    b_init: float = 0.0
    wd: Optional[float] = 0.0  # None => no weight_loss term at all


@dataclasses.dataclass
class MaxPool:
    name: str
    k: int = 2
    s: int = 2
    padding: str = "SAME"      # mnist_input.py:149-150,171-172


@dataclasses.dataclass
class LRN:
    name: str
    depth_radius: int = 4      # mnist_input.py:152-153,168-169
    bias: float = 1.0
    alpha: float = 0.001 / 9.0
    beta: float = 0.75


@dataclasses.dataclass
class Dense:
    name: str
    din: int
    dout: int
    relu: bool = True
    w_std: float = 0.04
    b_init: float = 0.1
    wd: Optional[float] = 0.0


Layer = Union[Conv, MaxPool, LRN, Dense]


@dataclasses.dataclass
class ModelSpec:
    name: str
    input_hw: Tuple[int, int]
    in_channels: int
    num_classes: int
    layers: List[Layer]

    # -- derived --------------------------------------------------------
    def shapes(self) -> List[Tuple[int, ...]]:
        """Per-layer output shape (per image): (H, W, C) or (D,)."""
        h, w = self.input_hw
        c = self.in_channels
        flat: Optional[int] = None
        out = []
        for L in self.layers:
            if isinstance(L, Conv):
                assert flat is None and c == L.cin, (L.name, c, L.cin)
                if L.padding == "VALID":
                    h, w = h - L.kh + 1, w - L.kw + 1
                c = L.cout
                out.append((h, w, c))
            elif isinstance(L, MaxPool):
                if L.padding == "SAME":
                    h, w = math.ceil(h / L.s), math.ceil(w / L.s)
                else:
                    h, w = (h - L.k) // L.s + 1, (w - L.k) // L.s + 1
                out.append((h, w, c))
            elif isinstance(L, LRN):
                out.append((h, w, c))
            elif isinstance(L, Dense):
                d = flat if flat is not None else h * w * c
                assert d == L.din, (L.name, d, L.din)
                flat = L.dout
                out.append((flat,))
            else:
                raise TypeError(L)
        return out

    def weights(self) -> List[Union[Conv, Dense]]:
        return [L for L in self.layers if isinstance(L, (Conv, Dense))]

    def param_shapes(self) -> List[Tuple[str, Tuple[int, ...]]]:
        """Trainable variables in creation order (mnist_input.py:137-205)."""
        res = []
        for L in self.weights():
            if isinstance(L, Conv):
                res.append((f"{L.name}/weights", (L.kh, L.kw, L.cin, L.cout)))
                res.append((f"{L.name}/biases", (L.cout,)))
            else:
                res.append((f"{L.name}/weights", (L.din, L.dout)))
                res.append((f"{L.name}/biases", (L.dout,)))
        return res

    def num_params(self) -> int:
        return sum(math.prod(s) for _, s in self.param_shapes())

    def flops_per_image(self) -> Tuple[float, float]:
        """(forward FLOP, forward+backward FLOP) per image, MAC = 2 FLOP."""
        h, w = self.input_hw
        fwd = 0.0
        bwd = 0.0
        shapes = self.shapes()
        first_w = True
        for L, s in zip(self.layers, shapes):
            if isinstance(L, Conv):
                macs = s[0] * s[1] * L.cout * L.kh * L.kw * L.cin
            elif isinstance(L, Dense):
                macs = L.din * L.dout
            else:
                continue
            fwd += 2 * macs
            bwd += 2 * macs * (1 if first_w else 2)   # first layer needs no dgrad
            first_w = False
        return fwd, fwd + bwd

    def loss_names(self) -> List[str]:
        """Entries of the reference's 'losses' collection (mnist_input.py:113,226)."""
        names = [f"{L.name}/weight_loss" for L in self.weights() if L.wd is not None]
        return names + ["cross_entropy"]
