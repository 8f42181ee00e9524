"""Hyper-parameter manager: the in-repo replacement for DLI's ``tf_parameter_mgr``.

The reference pulls every hyper-parameter and data list from an external
IBM Spectrum Conductor module (``main.py:35,38-40``; ``mnist_input.py:10,22-23,
47,50,261``; ``inference.py:63``).  That module is not in the repository; its API
surface is inferred from the call sites.  This module exposes
the same getters, backed by a YAML/JSON config file plus programmatic
overrides:

    getMaxSteps()            -> int
    getTestInterval()        -> int
    getTrainBatchSize()      -> int
    getLearningRateDecay()   -> float   (staircase decay factor)
    getBaseLearningRate()    -> float
    getTrainData()           -> list[str]
    getTestData()            -> list[str]
    getValData()             -> list[str]
    getOptimizer(lr)         -> OptimizerSpec

Defaults are the TF CIFAR-10 tutorial values that ``mnist_input.py`` mirrors
 — they are *chosen* defaults, not numbers the reference
publishes.  Data lists accept file paths / globs, ``synthetic://N`` or
``idx://<dir>`` / ``png://<dir>`` URIs (see ``data/``).

Unlike the reference (which evaluates the getters at import time,
``main.py:38-40``), values are read lazily so a ``--config`` flag parsed after
import still takes effect.
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Any, Dict, List, Optional, Union

DEFAULTS: Dict[str, Any] = {
    "max_steps": 1000,
    "test_interval": 100,
    "batch_size": 128,
    "base_lr": 0.1,
    "lr_decay": 0.1,
    "optimizer": "sgd",          # sgd | momentum | nesterov
    "momentum": 0.9,
    "train_data": ["synthetic://60000"],
    "test_data": ["synthetic://10000?seed=1"],
    "val_data": ["synthetic://10000?seed=2"],
}

ENV_VAR = "MNISTX_PARAMS"


@dataclasses.dataclass(frozen=True)
class OptimizerSpec:
    """What ``getOptimizer(lr)`` returns: enough to build the fused K9 update."""
    name: str            # "sgd" | "momentum"
    learning_rate: Any   # float, or a callable/step-schedule
    momentum: float = 0.0
    nesterov: bool = False


_config: Dict[str, Any] = {}
_loaded_from: Optional[str] = None


def _load_file(path: str) -> Dict[str, Any]:
    with open(path, "r") as f:
        text = f.read()
    if path.endswith((".yaml", ".yml")):
        import yaml
        data = yaml.safe_load(text) or {}
    else:
        data = json.loads(text)
    if not isinstance(data, dict):
        raise ValueError(f"config {path} must hold a mapping")
    return data


def _as_list(v: Union[str, List[str], None]) -> List[str]:
    if v is None:
        return []
    if isinstance(v, str):
        return [s for s in (p.strip() for p in v.split(",")) if s]
    return [str(x) for x in v]


def configure(source: Union[None, str, Dict[str, Any]] = None, **overrides: Any) -> None:
    """Load a config file/dict (replaces the current one) and apply overrides."""
    global _config, _loaded_from
    cfg: Dict[str, Any] = {}
    if source is None:
        env = os.environ.get(ENV_VAR)
        if env:
            cfg.update(_load_file(env))
            _loaded_from = env
    elif isinstance(source, str):
        cfg.update(_load_file(source))
        _loaded_from = source
    else:
        cfg.update(source)
        _loaded_from = "<dict>"
    for k, v in overrides.items():
        if v is not None:
            cfg[k] = v
    unknown = set(cfg) - set(DEFAULTS) - {"model", "in_channels", "seed", "weight_decay",
                                          "moving_average_decay", "num_epochs_per_decay",
                                          "examples_per_epoch"}
    if unknown:
        raise ValueError(f"unknown parameter(s) in config: {sorted(unknown)}")
    _config = cfg


def set_param(key: str, value: Any) -> None:
    _config[key] = value


def get(key: str, default: Any = None) -> Any:
    if key in _config:
        return _config[key]
    if key in DEFAULTS:
        return DEFAULTS[key]
    return default


def snapshot() -> Dict[str, Any]:
    out = dict(DEFAULTS)
    out.update(_config)
    return out


# --- the DLI getter surface --------------------------------
def getMaxSteps() -> int:
    return int(get("max_steps"))


def getTestInterval() -> int:
    return int(get("test_interval"))


def getTrainBatchSize() -> int:
    return int(get("batch_size"))


def getLearningRateDecay() -> float:
    return float(get("lr_decay"))


def getBaseLearningRate() -> float:
    return float(get("base_lr"))


def getTrainData() -> List[str]:
    return _as_list(get("train_data"))


def getTestData() -> List[str]:
    return _as_list(get("test_data"))


def getValData() -> List[str]:
    return _as_list(get("val_data"))


def getOptimizer(lr: Any) -> OptimizerSpec:
    """Config-driven optimizer choice (``mnist_input.py:261``)."""
    name = str(get("optimizer")).lower()
    mom = float(get("momentum"))
    if name in ("sgd", "gradientdescent", "gradient_descent"):
        return OptimizerSpec("sgd", lr, 0.0, False)
    if name == "momentum":
        return OptimizerSpec("momentum", lr, mom, False)
    if name == "nesterov":
        return OptimizerSpec("momentum", lr, mom, True)
    raise ValueError(f"unsupported optimizer {name!r} (sgd|momentum|nesterov)")


configure()
