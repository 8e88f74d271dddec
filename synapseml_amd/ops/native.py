"""Loader for the in-tree native modules (replaces the reference's
NativeLoader / LightGBMUtils.initializeNativeLibrary).

PyTorch is imported first when present: it bundles its own HIP runtime and
RCCL with the same SONAMEs, and loading it first guarantees one HIP runtime per
process. If a module is missing while a GPU is present this raises instead of
silently falling back (the driver checks which .so files a GPU run loaded).
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mods: dict = {}


def _import_torch_first() -> None:
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for the CPU path
        pass


def load(name: str):
    with _lock:
        if name in _mods:
            return _mods[name]
        _import_torch_first()
        try:
            m = importlib.import_module(f"synapseml_amd.{name}")
        except ImportError as e:
            script = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(__file__))), "tools",
                                  "build_native.py")
            if os.environ.get("SML_AUTOBUILD", "1") == "1" and os.path.exists(script):
                import subprocess
                import sys

                subprocess.run([sys.executable, script, "--only", name], check=True)
                m = importlib.import_module(f"synapseml_amd.{name}")
            else:
                raise ImportError(
                    f"native module synapseml_amd.{name} is not built; run `python tools/build_native.py`"
                ) from e
        _mods[name] = m
        return m


def gbdt():
    return load("_gbdt")


def gpu_available() -> bool:
    try:
        return bool(gbdt().gpu_available())
    except Exception:  # pragma: no cover
        return False
