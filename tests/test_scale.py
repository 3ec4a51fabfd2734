"""Replica actuator: the four /root/reference/scale/scale_test.go tests plus the behaviours
SURVEY.md §3.3 lists for scale.go:54-107 (clamping, int32, no-op contract, error texts)."""
import pytest

from kube_sqs_autoscaler_amd.utils.log import capture_logger


def mock_pod_autoscaler(nat, name, ns, max_, min_, init, up, down, lines=None):
    """NewMockPodAutoScaler (scale_test.go:85-115): two Deployments, one never scaled."""
    fake = nat.FakeDeployments(ns)
    fake.add("deploy", init)
    fake.add("deploy-no-scale", init)
    log = capture_logger(lines if lines is not None else [])
    p = nat.PodAutoScaler(fake, name, ns, max_, min_, up, down, log, nat.RealClock())
    return p, fake


def test_scale_up(nat):  # scale_test.go:14-33
    p, f = mock_pod_autoscaler(nat, "deploy", "namespace", 5, 1, 3, 1, 1)
    p.scale_up()
    assert f.replicas("deploy") == 4
    p.scale_up()
    assert f.replicas("deploy") == 5
    p.scale_up()  # no error at max
    assert f.replicas("deploy") == 5
    assert f.replicas("deploy-no-scale") == 3


def test_scale_up_with_scaling_pod_num(nat):  # scale_test.go:35-49
    p, f = mock_pod_autoscaler(nat, "deploy", "namespace", 10, 1, 3, 5, 5)
    p.scale_up()
    assert f.replicas("deploy") == 8
    p.scale_up()
    assert f.replicas("deploy") == 10


def test_scale_down(nat):  # scale_test.go:51-68
    p, f = mock_pod_autoscaler(nat, "deploy", "namespace", 5, 1, 3, 1, 1)
    p.scale_down()
    assert f.replicas("deploy") == 2
    p.scale_down()
    assert f.replicas("deploy") == 1
    p.scale_down()
    assert f.replicas("deploy") == 1


def test_scale_down_with_scaling_pod_num(nat):  # scale_test.go:70-83
    p, f = mock_pod_autoscaler(nat, "deploy", "namespace", 10, 1, 8, 5, 5)
    p.scale_down()
    assert f.replicas("deploy") == 3
    p.scale_down()
    assert f.replicas("deploy") == 1


def test_log_messages(nat):
    lines = []
    p, f = mock_pod_autoscaler(nat, "deploy", "namespace", 4, 3, 3, 1, 1, lines)
    p.scale_up()
    p.scale_up()
    p.scale_down()
    p.scale_down()
    msgs = [l.split('msg="')[1].rstrip('"') for l in lines]
    assert msgs == ["Scale up successful. Replicas: 4", "More than max pods running. No scale up. Replicas: 4",
                    "Scale down successful. Replicas: 3", "Less than min pods running. No scale down. Replicas: 3"]


def test_noop_span_and_write_span(nat):
    p, f = mock_pod_autoscaler(nat, "deploy", "namespace", 5, 1, 5, 1, 1)
    s = p.scale_up()
    assert s.read and not s.wrote and s.before == s.after == 5 and f.updates() == 0
    s = p.scale_down()
    assert s.wrote and (s.before, s.after) == (5, 4) and f.updates() == 1


def test_asymmetric_clamp_above_max_and_below_min(nat):
    # cur > max: ScaleUp no-ops, ScaleDown subtracts and clamps only at min
    p, f = mock_pod_autoscaler(nat, "deploy", "namespace", 5, 1, 9, 1, 1)
    p.scale_up()
    assert f.replicas("deploy") == 9
    p.scale_down()
    assert f.replicas("deploy") == 8
    # cur < min: ScaleUp adds a step, no snap to min
    p, f = mock_pod_autoscaler(nat, "deploy", "namespace", 10, 5, 1, 1, 1)
    p.scale_up()
    assert f.replicas("deploy") == 2
    p.scale_down()
    assert f.replicas("deploy") == 2


def test_int32_wraparound_like_go(nat):
    # nextReplicas := *cur + int32(ScaleUpPods) wraps in int32, then `> int32(Max)` fails
    p, f = mock_pod_autoscaler(nat, "deploy", "namespace", 2**31 - 1, 1, 2**31 - 10, 100, 1)
    p.scale_up()
    assert f.replicas("deploy") == nat.go_int32(2**31 - 10 + 100)
    # max given as a 64-bit int is truncated by int32(p.Max)
    p, f = mock_pod_autoscaler(nat, "deploy", "namespace", 2**32 + 3, 1, 1, 5, 1)
    p.scale_up()
    assert f.replicas("deploy") == 3


def test_error_wrapping(nat):
    p, f = mock_pod_autoscaler(nat, "deploy", "namespace", 5, 1, 3, 1, 1)
    f.fail_next_get(1, "connection refused")
    with pytest.raises(nat.NativeError, match="^Failed to get deployment from kube server, no scale up occurred: connection refused$"):
        p.scale_up()
    f.fail_next_update(1, "etcdserver: request timed out")
    with pytest.raises(nat.NativeError, match="^Failed to scale down: etcdserver: request timed out$"):
        p.scale_down()
    assert f.replicas("deploy") == 3
    f.conflict_next(1)
    with pytest.raises(nat.NativeError, match="the object has been modified"):
        p.scale_up()
    p2, _ = mock_pod_autoscaler(nat, "missing", "namespace", 5, 1, 3, 1, 1)
    with pytest.raises(nat.NativeError, match='no scale down occurred: deployments.apps "missing" not found'):
        p2.scale_down()


def test_deployment_without_replicas_is_an_error_not_a_crash(nat):
    fake = nat.FakeDeployments("ns")
    fake.add_without_replicas("d")
    p = nat.PodAutoScaler(fake, "d", "ns", 5, 1, 1, 1, capture_logger([]), nat.RealClock())
    with pytest.raises(nat.NativeError, match="no spec.replicas"):
        p.scale_up()
