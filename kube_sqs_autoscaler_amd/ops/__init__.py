"""Native extension loading.

Two in-tree artifacts back the framework (built by :mod:`kube_sqs_autoscaler_amd.ops.build`):

* ``_ksa_native`` -- the C++ runtime: control loop (the reference's ``Run``,
  /root/reference/main.go:35-80), SQS client (/root/reference/sqs/sqs.go), Deployment actuator
  (/root/reference/scale/scale.go), SigV4, HTTP/TLS transport and the localhost fakes.
* ``libksa_gpu.so`` -- the gfx950 HIP node probe (see :mod:`.gpu`).

``native()`` builds the extension on first use when it is missing or stale (a few seconds of
g++), and fails loudly if it cannot: there is no pure-Python fallback of the hot path.
"""
from __future__ import annotations

import importlib
import os
import threading
from types import ModuleType

_lock = threading.Lock()
_mod: ModuleType | None = None


class NativeUnavailable(RuntimeError):
    """The C++ runtime could not be built or imported."""


def _sources_present() -> bool:
    from pathlib import Path

    return (Path(__file__).resolve().parents[2] / "csrc" / "core").is_dir()


def native() -> ModuleType:
    """Returns the ``_ksa_native`` module, building it in-tree if needed."""
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        # An installed copy (wheel) ships the built module and no csrc/: nothing to build.
        if os.environ.get("KSA_NO_AUTOBUILD") != "1" and _sources_present():
            from . import build

            try:
                build.build_native(verbose=False)
            except Exception as e:  # pragma: no cover - toolchain failure
                raise NativeUnavailable(f"failed to build the native runtime: {e}") from e
        try:
            _mod = importlib.import_module("kube_sqs_autoscaler_amd.ops._ksa_native")
        except ImportError as e:  # pragma: no cover
            raise NativeUnavailable(f"cannot import the native runtime: {e}") from e
        return _mod


def native_path() -> str:
    return native().__file__
