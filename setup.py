"""Packaging (the reference's go.mod / `go build`, /root/reference/go.mod, Makefile:12-13).

``pip install .`` / ``pip wheel .`` compile the C++ runtime (csrc/ -> ops/_ksa_native) and, when
hipcc is present, the gfx950 library (ops/libksa_gpu.so) in-tree first, then ship both inside the
package, so an installed copy never needs the sources or a compiler at run time.
"""
import os
import sys

from setuptools import setup
from setuptools.command.build_py import build_py
from setuptools.dist import Distribution

ROOT = os.path.dirname(os.path.abspath(__file__))


class BuildWithNative(build_py):
    def run(self):
        sys.path.insert(0, ROOT)
        from kube_sqs_autoscaler_amd.ops import build

        build.build_native()
        try:
            build.build_gpu_probe()
        except RuntimeError as e:  # no ROCm toolchain: the control loop needs no GPU code
            print(f"[setup] skipping the gfx950 library: {e}")
        super().run()


class BinaryDistribution(Distribution):
    """The wheel carries a CPython extension: tag it for this interpreter and platform."""

    def has_ext_modules(self):
        return True


setup(
    name="kube-sqs-autoscaler-amd",
    version="0.1.0",
    description="SQS queue-depth autoscaler for Kubernetes GPU-worker Deployments on AMD Instinct MI355X nodes",
    license="MIT",
    python_requires=">=3.10",
    install_requires=["PyYAML>=5.4"],  # /metrics writes the Prometheus text format itself
    extras_require={"test": ["pytest>=7", "pytest-timeout", "hypothesis"], "bench": ["torch", "numpy"],
                    "tune": ["numpy"]},
    entry_points={"console_scripts": ["kube-sqs-autoscaler = kube_sqs_autoscaler_amd.cli:main_entry"]},
    packages=[
        "kube_sqs_autoscaler_amd", "kube_sqs_autoscaler_amd.bench", "kube_sqs_autoscaler_amd.kube",
        "kube_sqs_autoscaler_amd.models", "kube_sqs_autoscaler_amd.ops", "kube_sqs_autoscaler_amd.parallel",
        "kube_sqs_autoscaler_amd.sqs", "kube_sqs_autoscaler_amd.tune", "kube_sqs_autoscaler_amd.utils",
    ],
    package_data={"kube_sqs_autoscaler_amd": ["ops/*.so"]},
    cmdclass={"build_py": BuildWithNative},
    distclass=BinaryDistribution,
)
