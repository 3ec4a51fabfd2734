"""logrus TextFormatter compatibility (reference logs via logrus defaults, main.go:13)."""
from kube_sqs_autoscaler_amd.utils.log import capture_logger

T = 1700000000 * 10**9


def test_text_format_matches_logrus(nat):
    l = nat.Logger()
    assert l.format("info", "Found 3 messages in the queue", [], T) == \
        'time="2023-11-14T22:13:20Z" level=info msg="Found 3 messages in the queue"'
    assert l.format("info", "Waiting for cool down, skipping scale up ", [], T).endswith(
        'msg="Waiting for cool down, skipping scale up "')
    assert l.format("warning", "x", [], T) == 'time="2023-11-14T22:13:20Z" level=warning msg=x'
    # extra fields sorted by key, quoted only when needed (logrus needsQuoting)
    assert l.format("error", "e", [("queue", "https://a/b"), ("deployment", "ns/d")], T) == \
        'time="2023-11-14T22:13:20Z" level=error msg=e deployment=ns/d queue="https://a/b"'


def test_needs_quoting(nat):
    assert not nat.logrus_needs_quoting("abc-DEF_0.9/x@y^z+")
    for s in ("a b", "a:b", "a=b", '"', "", "é"):
        assert nat.logrus_needs_quoting(s) or s == ""


def test_json_format(nat):
    l = nat.Logger()
    l.set_format("json")
    assert l.format("info", "hi", [("a", "b")], T) == '{"a":"b","level":"info","msg":"hi","time":"2023-11-14T22:13:20Z"}'


def test_levels_filter(nat):
    lines = []
    l = capture_logger(lines, level="error")
    l.log("info", "dropped")
    l.log("error", "kept")
    assert len(lines) == 1 and "kept" in lines[0]


def test_with_fields_shares_sink(nat):
    lines = []
    base = capture_logger(lines)
    child = base.with_fields([("queue", "q1")])
    child.log("info", "m")
    base.log("info", "n")
    assert "queue=q1" in lines[0] and "queue" not in lines[1]


def test_loop_log_catalogue(nat):
    """Every reference loop message, emitted by the native loop."""
    from kube_sqs_autoscaler_amd.models import oracle, parity, traces

    sc = traces.c2_step()
    sc.polls = 40
    lines = []
    parity.run_native(sc, log_sink=lines.append)
    msgs = {l.split('msg="', 1)[1].rsplit('"', 1)[0] if 'msg="' in l else l for l in lines}
    for m in ["Found 0 messages in the queue", "Found 200 messages in the queue",
              "Waiting for cool down, skipping scale up ", "Waiting for cool down, skipping scale down",
              "Scale up successful. Replicas: 2", "Scale down successful. Replicas: 7",
              "More than max pods running. No scale up. Replicas: 8",
              "Less than min pods running. No scale down. Replicas: 1"]:
        assert m in msgs, m
    lines.clear()
    parity.run_native(sc, faults=oracle.Faults(sqs={1}, up_get={12}, up_update={13}), log_sink=lines.append)
    text = "\n".join(lines)
    assert 'level=error msg="Failed to get SQS messages: Failed to get messages in SQS: injected SQS failure"' in text
    assert "Failed scaling up: Failed to get deployment from kube server, no scale up occurred: injected GET failure" in text
    assert "Failed scaling up: Failed to scale up: injected PUT failure" in text
