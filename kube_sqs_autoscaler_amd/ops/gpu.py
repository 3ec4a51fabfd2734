"""ctypes binding of the gfx950 node probe (``csrc/hip/gpu_probe.hip`` -> ``libksa_gpu.so``).

Not a reference capability (the reference has no GPU code). It backs the
``--gpu-aware-max`` extension: when the autoscaler runs on the 8x MI355X node it scales, it can
cap ``--max-pods`` at the number of GPUs that pass an HBM write/verify health check.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from pathlib import Path

_LIB: ctypes.CDLL | None = None


class GpuProbeError(RuntimeError):
    pass


class _Info(ctypes.Structure):
    _fields_ = [
        ("name", ctypes.c_char * 256),
        ("arch", ctypes.c_char * 64),
        ("compute_units", ctypes.c_int32),
        ("clock_khz", ctypes.c_int32),
        ("warp_size", ctypes.c_int32),
        ("pci_bus_id", ctypes.c_int32),
        ("pci_device_id", ctypes.c_int32),
        ("lds_bytes_per_block", ctypes.c_int32),
        ("total_mem_bytes", ctypes.c_int64),
        ("free_mem_bytes", ctypes.c_int64),
    ]


class _Health(ctypes.Structure):
    _fields_ = [
        ("bytes", ctypes.c_uint64),
        ("checksum", ctypes.c_uint64),
        ("expected_checksum", ctypes.c_uint64),
        ("mismatches", ctypes.c_uint64),
        ("fill_ms", ctypes.c_double),
        ("verify_ms", ctypes.c_double),
        ("write_gbps", ctypes.c_double),
        ("read_gbps", ctypes.c_double),
    ]


@dataclass
class GpuInfo:
    index: int
    name: str
    arch: str
    compute_units: int
    clock_khz: int
    wavefront_size: int
    pci_bus_id: int
    lds_bytes_per_block: int
    total_mem_bytes: int
    free_mem_bytes: int


@dataclass
class GpuHealth:
    index: int
    ok: bool
    bytes: int
    checksum: int
    expected_checksum: int
    mismatches: int
    fill_ms: float
    verify_ms: float
    write_gbps: float
    read_gbps: float


def lib_path() -> Path:
    """The in-tree gfx950 library; ``KSA_GPU_LIB`` points at another build (A/B kernel runs)."""
    override = os.environ.get("KSA_GPU_LIB")
    return Path(override) if override else Path(__file__).resolve().parent / "libksa_gpu.so"


def load(build_if_missing: bool = True) -> ctypes.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    p = lib_path()
    if not p.exists() and build_if_missing and os.environ.get("KSA_NO_AUTOBUILD") != "1":
        from . import build

        build.build_gpu_probe(verbose=False)
    if not p.exists():
        raise GpuProbeError(f"{p} is missing; run python -m kube_sqs_autoscaler_amd.ops.build")
    lib = ctypes.CDLL(str(p))
    lib.ksa_gpu_last_error.restype = ctypes.c_char_p
    lib.ksa_gpu_device_count.restype = ctypes.c_int
    lib.ksa_gpu_get_info.argtypes = [ctypes.c_int, ctypes.POINTER(_Info)]
    lib.ksa_gpu_get_info.restype = ctypes.c_int
    lib.ksa_gpu_health_check.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(_Health)]
    lib.ksa_gpu_health_check.restype = ctypes.c_int
    lib.ksa_gpu_health_check_ex.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(_Health)]
    lib.ksa_gpu_health_check_ex.restype = ctypes.c_int
    _LIB = lib
    return lib


def _err(lib: ctypes.CDLL) -> str:
    return (lib.ksa_gpu_last_error() or b"").decode(errors="replace")


def device_count() -> int:
    lib = load()
    n = lib.ksa_gpu_device_count()
    if n < 0:
        raise GpuProbeError(_err(lib))
    return n


def device_info(index: int) -> GpuInfo:
    lib = load()
    info = _Info()
    if lib.ksa_gpu_get_info(index, ctypes.byref(info)) != 0:
        raise GpuProbeError(_err(lib))
    return GpuInfo(
        index=index,
        name=info.name.decode(errors="replace"),
        arch=info.arch.decode(errors="replace"),
        compute_units=info.compute_units,
        clock_khz=info.clock_khz,
        wavefront_size=info.warp_size,
        pci_bus_id=info.pci_bus_id,
        lds_bytes_per_block=info.lds_bytes_per_block,
        total_mem_bytes=info.total_mem_bytes,
        free_mem_bytes=info.free_mem_bytes,
    )


def health_check(index: int, nbytes: int = 256 << 20, reps: int = 3) -> GpuHealth:
    """HBM fill + verify over ``nbytes`` on device ``index``: one warm-up, then best of ``reps``.

    Bandwidth figures are HBM figures only for buffers well past the 256 MiB Infinity Cache
    (use >= 1 GiB); the health verdict holds for any size.
    """
    lib = load()
    h = _Health()
    rc = lib.ksa_gpu_health_check_ex(index, nbytes, reps, ctypes.byref(h))
    if rc < 0:
        raise GpuProbeError(_err(lib))
    return GpuHealth(
        index=index,
        ok=rc == 0,
        bytes=h.bytes,
        checksum=h.checksum,
        expected_checksum=h.expected_checksum,
        mismatches=h.mismatches,
        fill_ms=h.fill_ms,
        verify_ms=h.verify_ms,
        write_gbps=h.write_gbps,
        read_gbps=h.read_gbps,
    )


def healthy_gpu_count(nbytes: int = 64 << 20) -> int:
    """Number of local GPUs that pass :func:`health_check` (0 when there is no GPU)."""
    n = device_count()
    return sum(1 for i in range(n) if health_check(i, nbytes, reps=1).ok)
