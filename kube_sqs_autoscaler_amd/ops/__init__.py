"""Native extension loading.

Two in-tree artifacts back the framework (built by :mod:`kube_sqs_autoscaler_amd.ops.build`):

* ``_ksa_native`` -- the C++ runtime: control loop (the reference's ``Run``,
  /root/reference/main.go:35-80), SQS client (/root/reference/sqs/sqs.go), Deployment actuator
  (/root/reference/scale/scale.go), SigV4, HTTP/TLS transport. The image ships this one.
* ``_ksa_fakes`` -- the native test doubles: localhost fake SQS / kube-apiserver endpoints and
  the in-memory fakes of the two API seams (the reference keeps its mocks in ``_test.go`` files,
  /root/reference/main_test.go:241-304, /root/reference/sqs/sqs_test.go:27-59). Tests, the
  benchmark and the parity harness load it with :func:`fakes`.
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
_fakes: ModuleType | None = None


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
                if not build.native_up_to_date():
                    build.build_native(verbose=False)
            except Exception as e:  # pragma: no cover - toolchain failure
                raise NativeUnavailable(f"failed to build the native runtime: {e}") from e
        try:
            _mod = importlib.import_module("kube_sqs_autoscaler_amd.ops._ksa_native")
        except ImportError as e:  # pragma: no cover
            raise NativeUnavailable(f"cannot import the native runtime: {e}") from e
        return _mod


def fakes() -> ModuleType:
    """Returns the ``_ksa_fakes`` module (test doubles), building it in-tree if needed. It
    registers subclasses of ``_ksa_native``'s seams, so the runtime is loaded first."""
    global _fakes
    if _fakes is not None:
        return _fakes
    if not native().HTTP_TIMING and _sources_present():
        # a dev tree running the image build (-DKSA_HTTP_TIMING=0): the attribution rows would
        # come out empty (an image has no sources and no fakes: the import below says so)
        raise NativeUnavailable("the loaded _ksa_native is the image build (no HTTP timing, no test doubles); "
                                "rebuild the dev module: python -m kube_sqs_autoscaler_amd.ops.build")
    with _lock:
        if _fakes is not None:
            return _fakes
        if os.environ.get("KSA_NO_AUTOBUILD") != "1" and _sources_present():
            from . import build

            try:
                if not build.fakes_up_to_date():
                    build.build_fakes(verbose=False)
            except Exception as e:  # pragma: no cover - toolchain failure
                raise NativeUnavailable(f"failed to build the native fakes: {e}") from e
        try:
            _fakes = importlib.import_module("kube_sqs_autoscaler_amd.ops._ksa_fakes")
        except ImportError as e:
            raise NativeUnavailable(f"cannot import the native fakes (test builds only): {e}") from e
        return _fakes
