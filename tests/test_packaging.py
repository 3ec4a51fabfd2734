"""Packaging (the reference's go.mod + `go build`): setup.py must ship every subpackage, and the
built native module, so an installed wheel runs without csrc/ or a compiler."""
import ast
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup_kwargs():
    tree = ast.parse(open(os.path.join(ROOT, "setup.py")).read())
    call = next(n for n in ast.walk(tree) if isinstance(n, ast.Call) and getattr(n.func, "id", "") == "setup")
    return {kw.arg: kw.value for kw in call.keywords}


def test_every_subpackage_is_packaged():
    from setuptools import find_packages

    listed = set(ast.literal_eval(_setup_kwargs()["packages"]))
    assert listed == set(find_packages(ROOT, include=["kube_sqs_autoscaler_amd*"]))


def test_native_module_is_package_data_and_console_script_matches_reference_name():
    kw = _setup_kwargs()
    assert "ops/*.so" in ast.literal_eval(kw["package_data"])["kube_sqs_autoscaler_amd"]
    scripts = ast.literal_eval(kw["entry_points"])["console_scripts"]
    assert scripts == ["kube-sqs-autoscaler = kube_sqs_autoscaler_amd.cli:main_entry"]


def _docker_stages():
    stages = []
    for line in open(os.path.join(ROOT, "Dockerfile")):
        if line.startswith("FROM "):
            parts = line.split()
            stages.append({"base": parts[1], "name": parts[3] if len(parts) > 3 else "", "body": []})
        elif stages:
            stages[-1]["body"].append(line)
    return stages


def _code(stage):
    return [l for l in stage["body"] if l.strip() and not l.lstrip().startswith("#")]


def test_default_image_is_slim_and_no_runtime_stage_is_a_dev_image():
    """`docker build .` builds the last stage: the slim control-loop image. Only the GPU image's
    builder uses the ROCm dev image; the GPU image adds the HIP runtime package alone."""
    stages = _docker_stages()
    assert stages[-1]["name"] == "slim"
    runtime = [s for s in stages if not s["name"].endswith("builder")]
    assert all("dev" not in s["base"] for s in runtime)
    assert not any("pip" in l for s in runtime for l in _code(s))
    gpu = next(s for s in stages if s["name"] == "gpu")
    assert any("hip-runtime-amd" in l for l in gpu["body"])
    base = next(s for s in stages if s["name"] == "runtime")
    assert any("/kube-sqs-autoscaler /kube-sqs-autoscaler" in l for l in base["body"])  # the reference's command path
    assert all(s["base"] == "runtime" for s in stages if s["name"] in ("gpu", "slim"))


def test_slim_stage_chain_never_references_rocm():
    """The slim image and every stage it is built from or copies from (its builder included)
    use no ROCm image or package: a CPU-only control loop needs no multi-GB toolchain."""
    import re

    stages = {s["name"]: s for s in _docker_stages()}
    chain, todo = set(), ["slim"]
    while todo:
        name = todo.pop()
        if name in chain or name not in stages:
            continue
        chain.add(name)
        st = stages[name]
        todo.append(st["base"])
        todo += re.findall(r"--from=(\S+)", "".join(_code(st)))
    assert chain == {"slim", "runtime", "slim-builder"}, chain
    for name in chain:
        st = stages[name]
        assert "rocm" not in st["base"].lower(), name
        assert not any(re.search(r"rocm|hipcc|hip-runtime|offload-arch", l, re.I) for l in _code(st)), name
    # both builders ship the image runtime: timing compiled out, test doubles removed
    for name in ("slim-builder", "gpu-builder"):
        assert any("ops.build" in l and "--image" in l for l in _code(stages[name])), name


def test_docker_context_excludes_host_built_libraries():
    """COPY . /work must not carry a host-built .so (libksa_gpu.so, _ksa_fakes) into an image:
    the builders compile everything from source."""
    lines = [l.strip() for l in open(os.path.join(ROOT, ".dockerignore")) if l.strip() and not l.startswith("#")]
    assert "**/*.so" in lines and "build" in lines


def test_ci_workflow_runs_the_ci_gate():
    import yaml

    wf = yaml.safe_load(open(os.path.join(ROOT, ".github", "workflows", "ci.yml")))
    steps = [st.get("run", "") for st in wf["jobs"]["cpu"]["steps"]]
    assert any("make ci" in r for r in steps)
    image = [st.get("run", "") for st in wf["jobs"]["image"]["steps"]]
    assert any("docker build --target slim" in r for r in image)
    assert any("_ksa_fakes" in r for r in image)
    assert "make ci" in open(os.path.join(ROOT, "Makefile")).read() or "scripts/ci.sh" in open(os.path.join(ROOT, "Makefile")).read()


def test_module_up_to_date_check_needs_no_object_files(tmp_path, monkeypatch):
    """native()/fakes() rebuild only when the module is older than a source: a GPU box gets the
    built modules without build/ (gpurun ignores it), and several bench ranks starting at once
    must not all recompile a current module."""
    import time

    from kube_sqs_autoscaler_amd.ops import build

    so = tmp_path / "mod.so"
    so.write_bytes(b"")
    monkeypatch.setattr(build, "NATIVE_SO", so)
    monkeypatch.setattr(build, "FAKES_SO", so)
    monkeypatch.setattr(build, "BUILD", tmp_path / "no-build-dir")
    os.utime(so, (0, 0))
    assert not build.native_up_to_date() and not build.fakes_up_to_date()
    future = time.time() + 3600
    os.utime(so, (future, future))
    assert build.native_up_to_date() and build.fakes_up_to_date()
    so.unlink()
    assert not build.native_up_to_date()
