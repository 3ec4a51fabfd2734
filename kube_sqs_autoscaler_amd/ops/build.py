"""In-tree build of the native runtime and the gfx950 GPU probe.

Artifacts (git-ignored, but they travel to the GPU box with the gpurun snapshot):

* ``kube_sqs_autoscaler_amd/ops/_ksa_native<EXT_SUFFIX>`` -- pybind11 module linking the C++
  core in ``csrc/core`` (control loop, SigV4, HTTP/TLS client, SQS + Kubernetes clients)
  against OpenSSL. This is the production runtime the image ships.
* ``kube_sqs_autoscaler_amd/ops/_ksa_fakes<EXT_SUFFIX>`` -- the test doubles in ``csrc/fakes``
  (localhost fake SQS / kube-apiserver, their HTTP server, in-memory API fakes), linked against
  the core as a static archive (only what they use). Tests, the benchmark and the parity
  harness load it; the slim image does not contain it.
* ``kube_sqs_autoscaler_amd/ops/libksa_gpu.so`` -- ``hipcc --offload-arch=gfx950`` build of
  ``csrc/hip/gpu_probe.hip`` (GPU inventory + HBM health check), loaded with ctypes.
* ``build/native_tests[_asan|_tsan]`` -- host-only C++ test binaries (sanitizer builds).
* ``build/fuzz_wire`` -- libFuzzer + ASan/UBSan harness over every wire/plugin parser
  (``csrc/tests/fuzz_wire.cc``), built with ROCm's clang.

Objects are compiled in parallel and reused when neither the source nor any header under
``csrc/`` changed, so an incremental rebuild after touching one file takes seconds.

``--image`` builds what the container image ships instead: ``_ksa_native`` alone, with the
per-request HTTP timing diagnostics compiled out (``-DKSA_HTTP_TIMING=0``), and removes
``_ksa_fakes`` from the package (Dockerfile).

Usage: ``python -m kube_sqs_autoscaler_amd.ops.build [--no-hip] [--sanitizers] [--fuzz] [--image]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
import threading
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
CSRC = ROOT / "csrc"
OPS = Path(__file__).resolve().parent
BUILD = ROOT / "build"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
NATIVE_SO = OPS / f"_ksa_native{EXT_SUFFIX}"
FAKES_SO = OPS / f"_ksa_fakes{EXT_SUFFIX}"
# Written next to the in-tree _ksa_native by build_image_runtime (the timing-less image build);
# removed by build_native. Its presence makes native_up_to_date() false, so a dev tree that ran
# `build --image` gets the release module back on the next native() instead of running tests and
# benchmarks without HTTP timing.
IMAGE_STAMP = OPS / "_ksa_native.image-build"
GPU_SO = OPS / "libksa_gpu.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")
CLANGXX = os.environ.get("FUZZ_CXX", "/opt/rocm/llvm/bin/clang++")
GPU_ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]

CXXFLAGS = ["-std=c++17", "-O2", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter", "-Werror=misleading-indentation",
            "-Werror=return-type", "-pthread"]
LIBS = ["-lssl", "-lcrypto", "-pthread"]


def _core_sources() -> list[Path]:
    return sorted((CSRC / "core").glob("*.cc"))


def _fakes_sources() -> list[Path]:
    return sorted((CSRC / "fakes").glob("*.cc"))


def _newest_header() -> float:
    hs = list(CSRC.rglob("*.h"))  # includes csrc/sim/policy_sim.h
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _stale(target: Path, deps: list[Path], header_mtime: float) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps) or header_mtime > t


def _private(path: Path) -> Path:
    """A per-process, per-thread temporary name next to `path` (then os.replace'd onto it)."""
    return path.with_name(f"{path.name}.{os.getpid()}.{threading.get_ident()}.tmp")


def _run(cmd: list[str]) -> None:
    proc = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"command failed ({proc.returncode}): {' '.join(cmd)}\n{proc.stdout}{proc.stderr}")


def _compile_objects(variant: str, extra: list[str], sources: list[Path], jobs: int, cxx: str = "") -> list[Path]:
    objdir = BUILD / f"obj-{variant}"
    objdir.mkdir(parents=True, exist_ok=True)
    hm = _newest_header()
    todo, objs = [], []
    for src in sources:
        obj = objdir / (src.stem + ".o")
        objs.append(obj)
        if _stale(obj, [src], hm):
            todo.append((obj, [cxx or CXX, *CXXFLAGS, *extra, "-c", str(src), "-o"]))
    if todo:
        def compile_one(obj: Path, cmd: list[str]) -> None:
            # to a private name, then renamed: concurrent builds (test workers) never see a
            # half-written object
            tmp = _private(obj)
            _run(cmd + [str(tmp)])
            os.replace(tmp, obj)

        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for f in [ex.submit(compile_one, o, c) for o, c in todo]:
                f.result()
    return objs


RELEASE_FLAGS = ["-fvisibility=hidden"]


IMAGE_FLAGS = RELEASE_FLAGS + ["-DKSA_HTTP_TIMING=0"]


def _binding_object(name: str, variant: str = "release", flags: list[str] = RELEASE_FLAGS) -> Path:
    import pybind11

    src = CSRC / "bindings" / f"{name}.cc"
    obj = BUILD / f"obj-{variant}" / f"{name}.o"
    obj.parent.mkdir(parents=True, exist_ok=True)
    if _stale(obj, [src], _newest_header()):
        tmp = _private(obj)
        _run([CXX, *CXXFLAGS, *flags, f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
              "-c", str(src), "-o", str(tmp)])
        os.replace(tmp, obj)
    return obj


def _link(out: Path, inputs: list[Path], verbose: bool) -> None:
    if _stale(out, inputs, 0.0):
        tmp = _private(out)
        _run([CXX, "-shared", "-o", str(tmp), *map(str, inputs), *LIBS])
        os.replace(tmp, out)
        if verbose:
            print(f"[build] linked {out.relative_to(ROOT)}")


def _newest_source(dirs: list[Path], files: list[Path]) -> float:
    paths = [p for d in dirs for p in d.rglob("*") if p.suffix in (".cc", ".h")] + files
    return max((p.stat().st_mtime for p in paths), default=0.0)


def native_up_to_date() -> bool:
    """The in-tree ``_ksa_native`` is newer than every source it is built from. Decided on the
    module and the sources alone, not the object files: ``build/`` does not travel with the tree
    (a GPU box gets the built module and no objects), and a process there must not recompile a
    module that is current -- least of all several ranks at once."""
    return NATIVE_SO.exists() and not IMAGE_STAMP.exists() and NATIVE_SO.stat().st_mtime >= _newest_source(
        [CSRC / "core", CSRC / "sim"], [CSRC / "bindings" / "module.cc"])


def fakes_up_to_date() -> bool:
    """:func:`native_up_to_date` for ``_ksa_fakes`` (the fakes and the core they link)."""
    return FAKES_SO.exists() and FAKES_SO.stat().st_mtime >= _newest_source(
        [CSRC / "core", CSRC / "sim", CSRC / "fakes"], [CSRC / "bindings" / "fakes_module.cc"])


def build_native(jobs: int = 8, verbose: bool = True) -> Path:
    """Builds the production pybind11 extension in place; returns its path."""
    core = _compile_objects("release", RELEASE_FLAGS, _core_sources(), jobs)
    _link(NATIVE_SO, core + [_binding_object("module")], verbose)
    IMAGE_STAMP.unlink(missing_ok=True)
    return NATIVE_SO


def build_image_runtime(jobs: int = 8, verbose: bool = True, out: Path = NATIVE_SO) -> Path:
    """The image's runtime: ``_ksa_native`` with the HTTP timing diagnostics compiled out, and no
    ``_ksa_fakes`` next to it. By default replaces the in-tree module and removes the in-tree
    ``_ksa_fakes`` (run it last, in the image builder); ``out`` elsewhere leaves both alone."""
    core = _compile_objects("image", IMAGE_FLAGS, _core_sources(), jobs)
    inputs = core + [_binding_object("module", "image", IMAGE_FLAGS)]
    tmp = _private(out)
    _run([CXX, "-shared", "-o", str(tmp), *map(str, inputs), *LIBS])
    os.replace(tmp, out)
    if out == NATIVE_SO:
        FAKES_SO.unlink(missing_ok=True)
        IMAGE_STAMP.write_text("-DKSA_HTTP_TIMING=0\n")
    if verbose:
        print(f"[build] linked {out} (image: -DKSA_HTTP_TIMING=0, no _ksa_fakes)")
    return out


def build_fakes(jobs: int = 8, verbose: bool = True) -> Path:
    """Builds the test-doubles extension (``_ksa_fakes``) in place; returns its path. The core
    goes in as a static archive, so the module carries only the core objects the fakes use."""
    core = _compile_objects("release", RELEASE_FLAGS, _core_sources(), jobs)
    archive = BUILD / "obj-release" / "libksa_core.a"
    if _stale(archive, core, 0.0):
        tmp = _private(archive)
        _run(["ar", "rcs", str(tmp), *map(str, core)])
        os.replace(tmp, archive)
    fakes = _compile_objects("release", RELEASE_FLAGS, _fakes_sources(), jobs)
    _link(FAKES_SO, fakes + [_binding_object("fakes_module"), archive], verbose)
    return FAKES_SO


def build_gpu_probe(verbose: bool = True) -> Path | None:
    """Compiles the gfx950 kernels -- HBM probe + open- and closed-loop what-if sweeps -- into one .so
    (cross-compiles without a GPU)."""
    srcs = [CSRC / "hip" / "gpu_probe.hip", CSRC / "hip" / "policy_sweep.hip", CSRC / "hip" / "queue_sweep.hip"]
    deps = srcs + [CSRC / "sim" / "policy_sim.h", CSRC / "sim" / "queue_sim.h"]
    if not Path(HIPCC).exists() and shutil.which("hipcc") is None:
        raise RuntimeError("hipcc not found; cannot build the gfx950 kernels")
    hipcc = HIPCC if Path(HIPCC).exists() else "hipcc"
    if _stale(GPU_SO, deps, 0.0):
        tmp = GPU_SO.with_suffix(".tmp.so")
        _run([hipcc, f"--offload-arch={GPU_ARCH}", "-O3", "-std=c++17", "-Wall", "-Werror=unused-value",
              "-Werror=unused-result", "-shared", "-fPIC", *map(str, srcs), "-o", str(tmp)])
        os.replace(tmp, GPU_SO)
        if verbose:
            print(f"[build] hipcc --offload-arch={GPU_ARCH} -> {GPU_SO.relative_to(ROOT)}")
    return GPU_SO


def build_native_tests(sanitizer: str | None = None, jobs: int = 8) -> Path:
    """Host-only C++ unit-test binary; `sanitizer` in {None, 'asan', 'tsan'}."""
    flags = {
        None: ["-g"],
        "asan": ["-g", "-O1", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
        "tsan": ["-g", "-O1", "-fsanitize=thread"],
    }[sanitizer]
    variant = sanitizer or "test"
    srcs = _core_sources() + _fakes_sources() + [CSRC / "tests" / "native_tests.cc"]
    objs = _compile_objects(variant, flags, srcs, jobs)
    out = BUILD / ("native_tests" + (f"_{sanitizer}" if sanitizer else ""))
    if _stale(out, objs, 0.0):
        _run([CXX, *flags, "-o", str(out), *map(str, objs), *LIBS])
    return out


# Globals are left uninstrumented: ROCm clang registers some merged string literals twice under
# -O1 -g and aborts on a false ODR violation that ASAN_OPTIONS cannot switch off.
FUZZ_FLAGS = ["-g", "-O1", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
              "-mllvm", "-asan-globals=0"]


def build_fuzzer(jobs: int = 8) -> Path:
    """libFuzzer harness over the wire parsers (needs a clang with libFuzzer: ROCm's has it)."""
    if not Path(CLANGXX).exists() and shutil.which(CLANGXX) is None:
        raise RuntimeError(f"{CLANGXX} not found; cannot build the fuzzer")
    # the loop and the fake endpoints are not wire parsers (and fakes.cc trips a clang ODR false
    # positive); the fakes' HTTP server is a target (request framing)
    srcs = [p for p in _core_sources() if p.stem not in ("runner", "sweep")] + [CSRC / "fakes" / "http_server.cc",
                                                                                CSRC / "tests" / "fuzz_wire.cc"]
    objs = _compile_objects("fuzz", FUZZ_FLAGS + ["-fsanitize=fuzzer-no-link"], srcs, jobs, cxx=CLANGXX)
    out = BUILD / "fuzz_wire"
    if _stale(out, objs, 0.0):
        _run([CLANGXX, *FUZZ_FLAGS, "-fsanitize=fuzzer", "-o", str(out), *map(str, objs), *LIBS])
    return out


def build_all(hip: bool = True, jobs: int = 8) -> dict:
    out = {"native": str(build_native(jobs=jobs)), "fakes": str(build_fakes(jobs=jobs))}
    if hip:
        out["gpu_probe"] = str(build_gpu_probe())
    return out


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--no-hip", action="store_true", help="skip the gfx950 probe")
    ap.add_argument("--sanitizers", action="store_true", help="also build ASan/UBSan and TSan test binaries")
    ap.add_argument("--fuzz", action="store_true", help="also build the libFuzzer wire-parser harness")
    ap.add_argument("--image", action="store_true",
                    help="build the image's runtime only: _ksa_native without HTTP timing, _ksa_fakes removed")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    args = ap.parse_args(argv)
    if args.image:
        out = {"native": str(build_image_runtime(jobs=args.jobs))}
        if not args.no_hip:
            out["gpu_probe"] = str(build_gpu_probe())
        print(out)
        return 0
    print(build_all(hip=not args.no_hip, jobs=args.jobs))
    if args.sanitizers:
        for s in (None, "asan", "tsan"):
            print(build_native_tests(s, jobs=args.jobs))
    if args.fuzz:
        print(build_fuzzer(jobs=args.jobs))
    return 0


if __name__ == "__main__":
    sys.exit(main())
