import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: multi-second test")
    config.addinivalue_line("markers", "serial: timing-sensitive; skipped under pytest-xdist workers "
                                       "(CI runs them in a serial pass: scripts/ci.sh)")


def pytest_collection_modifyitems(config, items):
    if not os.environ.get("PYTEST_XDIST_WORKER"):
        return
    skip = pytest.mark.skip(reason="serial test: measures timing, so it runs only outside xdist (scripts/ci.sh)")
    for item in items:
        if "serial" in item.keywords:
            item.add_marker(skip)


class _RuntimeAndFakes:
    """One handle on the production runtime (_ksa_native) and the native test doubles
    (_ksa_fakes, a separate module the image does not ship): names resolve in the runtime first."""

    def __init__(self, runtime, doubles):
        self._runtime, self._doubles = runtime, doubles

    def __getattr__(self, name):
        try:
            return getattr(self._runtime, name)
        except AttributeError:
            return getattr(self._doubles, name)


@pytest.fixture(scope="session")
def nat():
    from kube_sqs_autoscaler_amd.ops import fakes, native

    return _RuntimeAndFakes(native(), fakes())
