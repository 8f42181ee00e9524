"""Model registry.

* ``reference_cnn`` — the reference's CIFAR-10-tutorial-style CNN, exact topology,
  init and weight decay of ``mnist_input.inference`` (``mnist_input.py:118-208``):
  conv5x5x32 → maxpool → LRN → conv5x5x64 → LRN → maxpool → FC1024 → FC192 → FC10.
  ``in_channels`` 3 reproduces the DLI 3-channel TFRecords (``mnist_input.py:13-15,
  134``); 1 is the BASELINE synthetic 28×28×1 configuration.
* ``lenet5`` — the model BASELINE.json names: conv5x5x6(SAME) → maxpool →
  conv5x5x16(VALID) → maxpool → FC120 → FC84 → FC10 with ReLU (modern LeNet-5).
  Not present in the reference; added for the BASELINE configs.
* ``mlp`` — 784→128→10, the BASELINE "single-process CPU plumbing" config.
"""
from __future__ import annotations

import math
from typing import Callable, Dict

from .spec import Conv, Dense, LRN, MaxPool, ModelSpec


def reference_cnn(in_channels: int = 3) -> ModelSpec:
    return ModelSpec(
        name="reference_cnn",
        input_hw=(28, 28),
        in_channels=in_channels,
        num_classes=10,
        layers=[
            Conv("conv1", 5, 5, in_channels, 32, "SAME", True, 5e-2, 0.0, 0.0),     # 136-145
            MaxPool("pool1"),                                                      # 149-150
            LRN("norm1"),                                                          # 152-153
            Conv("conv2", 5, 5, 32, 64, "SAME", True, 5e-2, 0.1, 0.0),             # 156-164
            LRN("norm2"),                                                          # 168-169
            MaxPool("pool2"),                                                      # 171-172
            Dense("local3", 7 * 7 * 64, 1024, True, 0.04, 0.1, 0.004),             # 175-184
            Dense("local4", 1024, 192, True, 0.04, 0.1, 0.004),                    # 188-193
            Dense("softmax_linear", 192, 10, False, 1 / 192.0, 0.0, 0.0),          # 200-205
        ],
    )


def lenet5(in_channels: int = 1) -> ModelSpec:
    he = lambda fan_in: math.sqrt(2.0 / fan_in)  # noqa: E731  (ReLU nets)
    return ModelSpec(
        name="lenet5",
        input_hw=(28, 28),
        in_channels=in_channels,
        num_classes=10,
        layers=[
            Conv("conv1", 5, 5, in_channels, 6, "SAME", True, he(25 * in_channels), 0.0, 0.0),
            MaxPool("pool1"),
            Conv("conv2", 5, 5, 6, 16, "VALID", True, he(150), 0.0, 0.0),
            MaxPool("pool2"),
            Dense("fc3", 400, 120, True, he(400), 0.0, 0.0),
            Dense("fc4", 120, 84, True, he(120), 0.0, 0.0),
            Dense("softmax_linear", 84, 10, False, 1 / 84.0, 0.0, 0.0),
        ],
    )


def mlp(in_channels: int = 1) -> ModelSpec:
    d = 28 * 28 * in_channels
    return ModelSpec(
        name="mlp",
        input_hw=(28, 28),
        in_channels=in_channels,
        num_classes=10,
        layers=[
            Dense("hidden", d, 128, True, math.sqrt(2.0 / d), 0.0, 0.0),
            Dense("softmax_linear", 128, 10, False, 1 / 128.0, 0.0, 0.0),
        ],
    )


MODELS: Dict[str, Callable[..., ModelSpec]] = {
    "reference_cnn": reference_cnn,
    "lenet5": lenet5,
    "mlp": mlp,
}


def get_model(name: str, in_channels: int | None = None) -> ModelSpec:
    if name not in MODELS:
        raise KeyError(f"unknown model {name!r}; choose from {sorted(MODELS)}")
    fn = MODELS[name]
    return fn() if in_channels is None else fn(in_channels)
