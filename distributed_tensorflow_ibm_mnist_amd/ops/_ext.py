"""Loader for the native extensions.

The HIP kernels are the compute path on MI355X: if ``_kernels`` is missing or
fails to load on a GPU machine we raise loudly instead of falling back to
PyTorch (a silent fallback would hide that the native code is not running).
"""
from __future__ import annotations

import importlib
import os
from types import ModuleType
from typing import Optional

_kernels: Optional[ModuleType] = None
_host: Optional[ModuleType] = None


class NativeExtensionError(RuntimeError):
    pass


def _import(name: str, builder) -> ModuleType:
    mod_name = f"distributed_tensorflow_ibm_mnist_amd.{name}"
    try:
        return importlib.import_module(mod_name)
    except ImportError as first:
        if os.environ.get("MNISTX_NO_AUTOBUILD"):
            raise NativeExtensionError(f"native extension {name} not built: {first}") from first
        try:
            builder()
        except Exception as e:  # build toolchain missing, compile error, ...
            raise NativeExtensionError(f"native extension {name} missing and build failed: {e}") from first
        importlib.invalidate_caches()
        return importlib.import_module(mod_name)


def kernels() -> ModuleType:
    """The HIP kernel extension (imports torch first so the HIP runtime is shared)."""
    global _kernels
    if _kernels is None:
        import torch  # noqa: F401  (load libamdhip64 / c10_hip before our .so)
        from .. import _build
        _kernels = _import("_kernels", lambda: _build.build_kernels(verbose=True))
    return _kernels


def host() -> ModuleType:
    """The host C++ runtime (TFRecord / crc32c / tensor bundle / IDX)."""
    global _host
    if _host is None:
        from .. import _build
        _host = _import("_host", lambda: _build.build_host(verbose=True))
    return _host
