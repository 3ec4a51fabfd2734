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
