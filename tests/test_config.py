"""Configuration model: reference flags, attribute-name rule (main.go:103-110), --queue specs."""
import pytest

from kube_sqs_autoscaler_amd.config import (
    DEFAULT_ATTRIBUTE_NAMES, MI355X_MAX_PODS, new_flag_set, parse_args, parse_attribute_names)
from kube_sqs_autoscaler_amd.utils.goflag import MINUTE, SECOND, FlagError

REFERENCE_FLAGS = {
    # name: (kind, default text)  -- /root/reference/main.go:83-97
    "poll-period": ("duration", "5s"), "scale-down-cool-down": ("duration", "30s"),
    "scale-up-cool-down": ("duration", "10s"), "scale-up-messages": ("int", "100"),
    "scale-down-messages": ("int", "10"), "scale-up-pods": ("int", "1"), "scale-down-pods": ("int", "1"),
    "max-pods": ("int", "8"), "min-pods": ("int", "1"), "aws-region": ("string", ""),
    "attribute-names": ("string", DEFAULT_ATTRIBUTE_NAMES), "sqs-queue-url": ("string", ""),
    "kubernetes-deployment": ("string", ""), "kubernetes-namespace": ("string", "default"),
}


def test_reference_flag_table():
    fs = new_flag_set()
    for name, (kind, default) in REFERENCE_FLAGS.items():
        f = fs.flags[name]
        assert (f.kind, f.default_text) == (kind, default), name


def test_reference_help_texts_verbatim():
    fs = new_flag_set()
    assert fs.flags["poll-period"].usage == "The interval in seconds for checking if scaling is required"
    assert fs.flags["scale-down-messages"].usage == "Number of messages required to scaling down"
    assert fs.flags["kubernetes-deployment"].usage == "Kubernetes Deployment to scale. This field is required"


def test_defaults():
    cfg = parse_args([], environ={})
    (t,) = cfg.targets
    assert t.poll_period_ns == 5 * SECOND and t.scale_up_cool_down_ns == 10 * SECOND
    assert t.scale_down_cool_down_ns == 30 * SECOND and t.max_pods == MI355X_MAX_PODS == 8
    assert t.attribute_names == DEFAULT_ATTRIBUTE_NAMES.split(",") and t.namespace == "default"
    assert cfg.scale_mode == "scale" and cfg.kube_config_path == ""


def test_readme_example_flags():
    # /root/reference/README.md:40-53
    cfg = parse_args([
        "--sqs-queue-url=https://sqs.us-east-1.amazonaws.com/123/q", "--kubernetes-deployment=worker",
        "--kubernetes-namespace=ml", "--aws-region=us-east-1", "--poll-period=5s", "--scale-down-cool-down=30s",
        "--scale-up-cool-down=5m", "--scale-up-messages=100", "--scale-down-messages=10", "--scale-up-pods=1",
        "--scale-down-pods=1", "--max-pods=5", "--min-pods=1", "--attribute-names=ApproximateNumberOfMessages",
    ], environ={"KUBE_CONFIG_PATH": "/k"})
    (t,) = cfg.targets
    assert t.scale_up_cool_down_ns == 5 * MINUTE and t.max_pods == 5 and t.namespace == "ml"
    assert t.attribute_names == ["ApproximateNumberOfMessages"] and cfg.kube_config_path == "/k"


@pytest.mark.parametrize("value,names", [
    (DEFAULT_ATTRIBUTE_NAMES, DEFAULT_ATTRIBUTE_NAMES.split(",")),
    ("ApproximateNumberOfMessages,ApproximateNumberOfMessagesNotVisible",
     ["ApproximateNumberOfMessages", "ApproximateNumberOfMessagesNotVisible"]),
    (" ApproximateNumberOfMessages , ApproximateNumberOfMessagesNotVisible ",
     ["ApproximateNumberOfMessages", "ApproximateNumberOfMessagesNotVisible"]),
    ("A,,B", ["A", "", "B"]),  # empty piece kept, like the reference (which then panics at sqs.go:58)
    ("", [""]),
    (DEFAULT_ATTRIBUTE_NAMES + " ", DEFAULT_ATTRIBUTE_NAMES.split(",")),  # differs as a string -> split+trim
    # strings.TrimSpace is unicode.IsSpace: U+001C..U+001F are kept (Python's str.strip drops
    # them), NEL / NBSP / U+3000 are trimmed
    ("A,\x1cB\x1c, C ", ["A", "\x1cB\x1c", "C"]),
    ("\x1f\x1eA", ["\x1f\x1eA"]),
    ("\u0085A ,　B \t", ["A", "B"]),
    ("​A", ["​A"]),  # ZERO WIDTH SPACE is not White_Space
])
def test_attribute_names_rule(value, names):
    assert parse_attribute_names(value) == names


def test_queue_specs():
    cfg = parse_args([
        "--max-pods=4",
        "--queue", "url=https://q/a,deployment=a,namespace=ns1",
        "--queue", "url=https://q/b,deployment=b,max-pods=8,scale-up-cool-down=1m,attribute-names=X|Y",
    ], environ={})
    assert [t.deployment for t in cfg.targets] == ["a", "b"]
    a, b = cfg.targets
    assert a.max_pods == 4 and a.namespace == "ns1" and b.max_pods == 8 and b.namespace == "default"
    assert b.scale_up_cool_down_ns == MINUTE and b.attribute_names == ["X", "Y"]


def test_queue_spec_plus_reference_form():
    cfg = parse_args(["--sqs-queue-url=u0", "--kubernetes-deployment=d0", "--queue=url=u1,deployment=d1"], environ={})
    assert [(t.queue_url, t.deployment) for t in cfg.targets] == [("u0", "d0"), ("u1", "d1")]


@pytest.mark.parametrize("argv", [
    ["--queue=deployment=x"], ["--queue=url=u,bogus=1"], ["--queue=url=u,max-pods=x"], ["--queue=url"],
    ["--scale-mode=watch"], ["--sqs-protocol=grpc"], ["--log-format=xml"], ["--gpu-aware-max=remote"],
    ["--busy-poll-budget=-1"], ["--busy-poll-budget=101"], ["--busy-poll-budget=NaN"], ["--busy-poll-budget=x"],
    ["--poll-prewarm=-1ms"],
])
def test_invalid_extension_values(argv):
    with pytest.raises(FlagError):
        parse_args(argv, environ={})
