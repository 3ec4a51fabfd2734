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


def test_tty_colored_layout_matches_logrus(nat):
    """logrus TextFormatter.printColored (the layout on a terminal): coloured 4-letter level,
    [seconds since start], message padded to 44 columns, coloured field keys."""
    log = nat.Logger()
    log.set_format("text-color")
    base = 1_700_000_000 * 10**9
    log.set_base_time(base)
    line = log.format("info", "Starting kube-sqs-autoscaler", [], base + 5 * 10**9 + 1)
    assert line == "\x1b[36mINFO\x1b[0m[0005] Starting kube-sqs-autoscaler" + " " * 16 + " "
    assert log.format("warning", "w", [], base).startswith("\x1b[33mWARN\x1b[0m[0000] w")
    assert log.format("error", "Failed scaling up: x", [], base).startswith("\x1b[31mERRO\x1b[0m[0000] ")
    assert log.format("debug", "d", [], base).startswith("\x1b[37mDEBU\x1b[0m")
    long = "m" * 50
    with_fields = log.format("info", long, [("queue", "a b"), ("deployment", "w")], base + 12 * 10**9)
    assert with_fields == f"\x1b[36mINFO\x1b[0m[0012] {long}  \x1b[36mdeployment\x1b[0m=w \x1b[36mqueue\x1b[0m=\"a b\""


def test_make_logger_picks_colors_on_a_tty(nat):
    import os
    import pty

    from kube_sqs_autoscaler_amd.utils.log import make_logger

    master, slave = pty.openpty()
    r, w = os.pipe()
    try:
        make_logger(fd=slave).log("info", "on a tty")
        make_logger(fd=w).log("info", "on a pipe")
        assert b"\x1b[36mINFO\x1b[0m" in os.read(master, 4096)
        assert os.read(r, 4096).startswith(b"time=")
    finally:
        for fd in (master, slave, r, w):
            os.close(fd)


def test_poll_lines_batched_in_order_over_the_wire(nat, tmp_path):
    """The production fd sink on a real clock: each poll's lines are held past the SQS answer
    and written while the replica write is on the wire or when the poll ends (LogBatch,
    csrc/core/log.h) -- same lines, same order as the reference (main.go:49,
    scale/scale.go:79), each stamped when it was logged."""
    import os

    from kube_sqs_autoscaler_amd.bench.latency import BenchEnv

    path = tmp_path / "loop.log"
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o600)
    env = BenchEnv(1, "scale", log_fd=fd)
    try:
        env.run(20)
    finally:
        env.close()
        os.close(fd)
    lines = path.read_text().splitlines()
    msgs = [l.split('msg="', 1)[1].rsplit('"', 1)[0] for l in lines]
    assert len(msgs) == 40
    for i in range(0, 40, 4):  # the trace alternates 200 / 0 messages
        assert msgs[i] == "Found 200 messages in the queue"
        assert msgs[i + 1].startswith("Scale up successful. Replicas: ")
        assert msgs[i + 2] == "Found 0 messages in the queue"
        assert msgs[i + 3].startswith("Scale down successful. Replicas: ")
    stamps = [l.split('time="', 1)[1].split('"', 1)[0] for l in lines]
    assert stamps == sorted(stamps)
