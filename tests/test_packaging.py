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


def test_default_image_is_slim_and_no_runtime_stage_is_a_dev_image():
    """`docker build .` builds the last stage: the slim control-loop image. Only the builder
    uses the ROCm dev image; the GPU image adds the HIP runtime package alone."""
    stages = _docker_stages()
    assert stages[-1]["name"] == "slim"
    runtime = [s for s in stages if s["name"] != "builder"]
    assert all("dev" not in s["base"] for s in runtime)
    assert not any("pip" in l for s in runtime for l in s["body"] if not l.lstrip().startswith("#"))
    gpu = next(s for s in stages if s["name"] == "gpu")
    assert any("hip-runtime-amd" in l for l in gpu["body"])
    base = next(s for s in stages if s["name"] == "base")
    assert any("/kube-sqs-autoscaler /kube-sqs-autoscaler" in l for l in base["body"])  # the reference's command path
    assert all(s["base"] == "base" for s in stages if s["name"] in ("gpu", "slim"))


def test_ci_workflow_runs_the_ci_gate():
    import yaml

    wf = yaml.safe_load(open(os.path.join(ROOT, ".github", "workflows", "ci.yml")))
    steps = [st.get("run", "") for st in wf["jobs"]["cpu"]["steps"]]
    assert any("make ci" in r for r in steps)
    assert "make ci" in open(os.path.join(ROOT, "Makefile")).read() or "scripts/ci.sh" in open(os.path.join(ROOT, "Makefile")).read()
