"""End-to-end over real sockets: native SQS/kube REST clients against the native fake servers."""
import pytest

from kube_sqs_autoscaler_amd.autoscaler import new_deployment_api, new_sqs_api
from kube_sqs_autoscaler_amd.kube.config import RestConfig
from kube_sqs_autoscaler_amd.sqs.credentials import static_provider
from kube_sqs_autoscaler_amd.utils.log import capture_logger

AKID, SECRET, REGION, TOKEN = "AKIDTEST", "secret/KEY", "eu-west-1", "tok-123"
ATTRS = {"ApproximateNumberOfMessages": "11", "ApproximateNumberOfMessagesDelayed": "2",
         "ApproximateNumberOfMessagesNotVisible": "5", "VisibilityTimeout": "30"}
NAMES = ["ApproximateNumberOfMessages", "ApproximateNumberOfMessagesDelayed", "ApproximateNumberOfMessagesNotVisible"]


@pytest.fixture
def sqs_server(nat):
    s = nat.FakeSqsServer()
    s.require_signature(AKID, SECRET, REGION)
    s.start()
    yield s
    s.stop()


@pytest.fixture
def kube_server(nat):
    k = nat.FakeKubeServer()
    k.require_token(TOKEN)
    k.start()
    k.add_deployment("ml", "worker", 3)
    yield k
    k.stop()


def sqs_client(nat, server, protocol="query", secret=SECRET, tls=None, retries=None):
    api = new_sqs_api(REGION, nat.RealClock(), endpoint=server.url, protocol=protocol,
                      credentials=static_provider(AKID, secret), tls=tls)
    url = f"{server.url}/123456789012/jobs"
    return nat.SqsClient(api, url, NAMES), api, url


@pytest.mark.parametrize("protocol", ["query", "json"])
def test_get_queue_attributes_signed(nat, sqs_server, protocol):
    c, api, url = sqs_client(nat, sqs_server, protocol)
    sqs_server.set_attributes(url, ATTRS)
    assert c.num_messages() == 18
    assert c.num_messages() == 18
    assert sqs_server.signature_failures() == 0
    assert sqs_server.connections() == 1  # keep-alive: one connection for both polls
    body = sqs_server.last_body()
    if protocol == "query":
        assert "Action=GetQueueAttributes" in body and "AttributeName.1=ApproximateNumberOfMessages" in body
        assert "Version=2012-11-05" in body
    else:
        assert '"AttributeNames"' in body and dict(sqs_server.last_headers())["X-Amz-Target"] == "AmazonSQS.GetQueueAttributes"


def test_bad_signature_is_rejected(nat, sqs_server):
    c, api, url = sqs_client(nat, sqs_server, secret="wrong")
    sqs_server.set_attributes(url, ATTRS)
    with pytest.raises(nat.NativeError, match="^Failed to get messages in SQS: SignatureDoesNotMatch"):
        c.num_messages()
    assert sqs_server.signature_failures() >= 1


def test_nonexistent_queue(nat, sqs_server):
    c, api, url = sqs_client(nat, sqs_server)
    with pytest.raises(nat.NativeError, match="NonExistentQueue"):
        c.num_messages()


def test_sdk_style_retries_on_5xx(nat, sqs_server):
    c, api, url = sqs_client(nat, sqs_server)
    sqs_server.set_attributes(url, ATTRS)
    sqs_server.inject(2, nat.InjectedFault(500, "oops"))
    assert c.num_messages() == 18  # DefaultRetryer: up to 3 retries
    assert api.stats()["retries"] == 2 and api.stats()["throttle_retries"] == 0
    sqs_server.inject(4, nat.InjectedFault(500, "down"))
    with pytest.raises(nat.NativeError):
        c.num_messages()
    assert api.stats()["retries"] == 5  # 3 more: DefaultRetryer.NumMaxRetries


@pytest.mark.parametrize("status,retried,throttled", [
    (503, True, True), (502, True, True), (504, True, True), (429, True, True),  # IsErrorThrottle
    (500, True, False),                                                          # IsErrorRetryable
    (501, False, False), (505, False, False), (403, False, False),                # final
])
def test_retry_classification_like_aws_sdk_go_v1(nat, sqs_server, status, retried, throttled):
    c, api, url = sqs_client(nat, sqs_server)
    sqs_server.set_attributes(url, ATTRS)
    sqs_server.inject(1, nat.InjectedFault(status, "x"))
    if retried:
        assert c.num_messages() == 18
    else:
        with pytest.raises(nat.NativeError):
            c.num_messages()
    st = api.stats()
    assert (st["retries"], st["throttle_retries"]) == (int(retried), int(throttled))


def test_no_retry_on_4xx(nat, sqs_server):
    c, api, url = sqs_client(nat, sqs_server)
    sqs_server.set_attributes(url, ATTRS)
    sqs_server.inject(1, nat.InjectedFault(400, "<ErrorResponse><Error><Code>InvalidAttributeName</Code><Message>bad</Message></Error></ErrorResponse>", "text/xml"))
    with pytest.raises(nat.NativeError, match="InvalidAttributeName"):
        c.num_messages()
    assert api.stats()["retries"] == 0


def test_reconnect_after_server_closed_idle_connection(nat, sqs_server):
    c, api, url = sqs_client(nat, sqs_server)
    sqs_server.set_attributes(url, ATTRS)
    assert c.num_messages() == 18
    sqs_server.drop_connections()
    assert c.num_messages() == 18
    assert sqs_server.connections() == 2


def test_missing_region_fails_every_poll(nat, sqs_server):
    api = new_sqs_api("", nat.RealClock(), credentials=static_provider(AKID, SECRET))
    c = nat.SqsClient(api, "https://sqs.example/1/q", NAMES)
    with pytest.raises(nat.NativeError, match="region"):
        c.num_messages()


def test_tls_sqs(nat):
    s = nat.FakeSqsServer()
    s.require_signature(AKID, SECRET, REGION)
    s.start("127.0.0.1", 0, True)
    try:
        tls = nat.TlsOptions()
        tls.ca_pem = s.cert_pem
        c, api, url = sqs_client(nat, s, tls=tls)
        assert url.startswith("https://")
        s.set_attributes(url, ATTRS)
        assert c.num_messages() == 18
        # untrusted CA -> verification failure
        c2, _, _ = sqs_client(nat, s, tls=nat.TlsOptions())
        with pytest.raises(nat.NativeError):
            c2.num_messages()
    finally:
        s.stop()


def scaler(nat, kube_server, mode, token=TOKEN, max_=5, min_=1, lines=None):
    api = new_deployment_api(RestConfig(host=kube_server.url, bearer_token=token), "ml", mode)
    log = capture_logger(lines if lines is not None else [])
    return nat.PodAutoScaler(api, "worker", "ml", max_, min_, 1, 1, log, nat.RealClock()), api


@pytest.mark.parametrize("mode,path,verb", [
    ("deployment", "/apis/apps/v1/namespaces/ml/deployments/worker", "PUT"),
    ("scale", "/apis/apps/v1/namespaces/ml/deployments/worker/scale", "PUT"),
    ("patch", "/apis/apps/v1/namespaces/ml/deployments/worker/scale", "PATCH"),
])
def test_kube_modes(nat, kube_server, mode, path, verb):
    p, api = scaler(nat, kube_server, mode)
    p.scale_up()
    assert kube_server.replicas("ml", "worker") == 4
    assert kube_server.last_method() == verb and kube_server.last_path() == path
    p.scale_down()
    p.scale_down()
    assert kube_server.replicas("ml", "worker") == 2
    assert kube_server.connections() == 1 and kube_server.auth_failures() == 0
    if mode == "deployment":
        import json

        body = json.loads(kube_server.last_body())
        assert body["kind"] == "Deployment" and body["spec"]["replicas"] == 2
        assert body["metadata"]["resourceVersion"]  # optimistic concurrency, like client-go Update


def test_kube_noop_does_not_write(nat, kube_server):
    p, api = scaler(nat, kube_server, "scale", max_=3)
    writes = kube_server.writes()
    p.scale_up()
    assert kube_server.writes() == writes and kube_server.replicas("ml", "worker") == 3


@pytest.mark.parametrize("mode", ["deployment", "scale", "patch"])
def test_kube_conflict_surfaces_as_error(nat, kube_server, mode):
    p, api = scaler(nat, kube_server, mode)
    kube_server.conflict_next(1)
    with pytest.raises(nat.NativeError, match="^Failed to scale up: .*the object has been modified"):
        p.scale_up()
    assert kube_server.replicas("ml", "worker") == 3
    p.scale_up()  # next poll retries with a fresh GET
    assert kube_server.replicas("ml", "worker") == 4


def test_kube_unauthorized(nat, kube_server):
    p, api = scaler(nat, kube_server, "scale", token="nope")
    with pytest.raises(nat.NativeError, match="no scale up occurred: Unauthorized"):
        p.scale_up()
    assert kube_server.auth_failures() == 1


def test_kube_not_found_and_5xx(nat, kube_server):
    api = new_deployment_api(RestConfig(host=kube_server.url, bearer_token=TOKEN), "ml", "scale")
    p = nat.PodAutoScaler(api, "ghost", "ml", 5, 1, 1, 1, capture_logger([]), nat.RealClock())
    with pytest.raises(nat.NativeError, match="not found"):
        p.scale_up()
    p2, _ = scaler(nat, kube_server, "scale")
    kube_server.inject(1, nat.InjectedFault(500, "boom"))
    with pytest.raises(nat.NativeError, match="no scale up occurred"):
        p2.scale_up()


def test_kube_tls_with_ca(nat):
    k = nat.FakeKubeServer()
    k.require_token(TOKEN)
    k.start("127.0.0.1", 0, True)
    try:
        k.add_deployment("ml", "worker", 1)
        api = new_deployment_api(RestConfig(host=k.url, bearer_token=TOKEN, ca_pem=k.cert_pem), "ml", "scale")
        p = nat.PodAutoScaler(api, "worker", "ml", 5, 1, 1, 1, capture_logger([]), nat.RealClock())
        p.scale_up()
        assert k.replicas("ml", "worker") == 2
    finally:
        k.stop()


def test_full_loop_over_the_wire(nat, sqs_server, kube_server):
    """Runner + real clients: scale up under backlog, down when drained (C2-shaped)."""
    c, _, url = sqs_client(nat, sqs_server)
    p, _ = scaler(nat, kube_server, "scale", max_=5)
    cfg = nat.LoopConfig()
    cfg.poll_period_ns = 0
    cfg.scale_up_cool_down_ns = 0
    cfg.scale_down_cool_down_ns = 0
    lines = []
    r = nat.Runner(cfg, c, p, nat.RealClock(), capture_logger(lines))
    r.arm()
    sqs_server.set_attributes(url, {n: "100" for n in NAMES})
    recs = r.steps(4)
    assert [x["up"] for x in recs] == ["scaled", "scaled", "noop", "noop"]
    assert kube_server.replicas("ml", "worker") == 5
    sqs_server.set_attributes(url, {n: "0" for n in NAMES})
    recs = r.steps(5)
    assert [x["down"] for x in recs] == ["scaled"] * 4 + ["noop"]
    assert kube_server.replicas("ml", "worker") == 1
    assert all(x["patch_latency_ns"] > 0 for x in recs[:4])
    st = r.stats()
    assert st["scale_ups"] == 2 and st["scale_downs"] == 4 and st["polls"] == 9


@pytest.mark.parametrize("mode", ["deployment", "scale", "patch"])
def test_prefetched_get_is_consumed(nat, kube_server, mode):
    p, api = scaler(nat, kube_server, mode)
    gets = kube_server.gets()
    assert p.prefetch()
    span = p.scale_up()
    assert span.used_prefetch and not span.refetched and span.wrote
    assert kube_server.gets() == gets + 1  # no second GET
    assert kube_server.replicas("ml", "worker") == 4


def test_unused_prefetch_is_drained(nat, kube_server):
    p, api = scaler(nat, kube_server, "scale")
    assert p.prefetch()
    p.discard_prefetch()
    p.scale_down()  # the connection is still in sync
    assert kube_server.replicas("ml", "worker") == 2 and kube_server.connections() == 1


@pytest.mark.parametrize("mode", ["deployment", "scale", "patch"])
def test_stale_prefetch_falls_back_to_fresh_read(nat, kube_server, mode):
    """A write conflict on the prefetched object re-reads and retries once (the reference's
    GET-after-poll); the caller sees a success, not a 409."""
    p, api = scaler(nat, kube_server, mode)
    kube_server.conflict_next(1)  # a concurrent writer right after the prefetched GET
    assert p.prefetch()
    span = p.scale_up()
    assert span.used_prefetch and span.refetched and span.wrote
    assert kube_server.replicas("ml", "worker") == 4
    assert kube_server.conflicts() == 1


def test_stale_prefetch_reevaluates_bounds(nat, kube_server):
    """After a conflict the decision is re-made on the fresh object (e.g. now at max -> no-op)."""
    import time

    p, api = scaler(nat, kube_server, "scale", max_=5)
    gets = kube_server.gets()
    assert p.prefetch()  # sees 3
    while kube_server.gets() == gets:  # the server has answered the pipelined GET
        time.sleep(0.001)
    kube_server.set_replicas("ml", "worker", 5)  # someone scaled to max meanwhile
    span = p.scale_up()
    assert span.refetched and not span.wrote
    assert kube_server.replicas("ml", "worker") == 5


def test_failed_prefetch_falls_back(nat, kube_server):
    p, api = scaler(nat, kube_server, "scale")
    kube_server.inject(1, nat.InjectedFault(500, "flaky"))
    assert p.prefetch()
    span = p.scale_up()  # the failed speculative GET is not reported; a fresh GET is made
    assert not span.used_prefetch and span.wrote
    assert kube_server.replicas("ml", "worker") == 4


def test_full_loop_pipelined_over_the_wire(nat, sqs_server, kube_server):
    c, _, url = sqs_client(nat, sqs_server)
    p, _ = scaler(nat, kube_server, "scale", max_=5)
    cfg = nat.LoopConfig()
    cfg.poll_period_ns = 0
    cfg.scale_up_cool_down_ns = 0
    cfg.scale_down_cool_down_ns = 0
    cfg.prefetch = True
    r = nat.Runner(cfg, c, p, nat.RealClock(), capture_logger([]))
    r.arm()
    p.warm()  # what --poll-prewarm does before a poll: the pipelined GET itself never dials
    sqs_server.set_attributes(url, {n: "100" for n in NAMES})
    recs = r.steps(4)
    assert [x["up"] for x in recs] == ["scaled", "scaled", "noop", "noop"] and all(x["prefetched"] for x in recs)
    sqs_server.set_attributes(url, {n: "10" for n in NAMES})  # 30 messages: dead band
    band = r.steps(3)
    # the first dead-band poll still predicted an up (its prefetch is drained unused); the
    # next two know the depth is in the dead band and send nothing, as the reference
    assert [x["prefetched"] for x in band] == [True, False, False] and [x["gets"] for x in band] == [1, 0, 0]
    sqs_server.set_attributes(url, {n: "0" for n in NAMES})
    recs = r.steps(5)
    assert [x["down"] for x in recs] == ["scaled"] * 4 + ["noop"]
    # the first drained poll reads synchronously (dead-band depth predicted nothing)
    assert [x["prefetched"] for x in recs] == [False] + [True] * 4 and all(x["gets"] == 1 for x in recs)
    assert kube_server.replicas("ml", "worker") == 1 and kube_server.connections() == 1
    # the reference reads on the 4 + 5 polls that act; the gate adds the one mispredicted poll
    assert kube_server.gets() == 10 and r.stats()["apiserver_reads"] == 10


def test_idle_queue_sends_no_speculative_gets(nat, sqs_server, kube_server):
    """C1-shaped idle queue (empty, replicas at min): with --pipeline-reads the apiserver sees
    exactly the reference's reads -- one GET per scale-down cool-down expiry (the no-op at min,
    /root/reference/scale/scale.go:82-92) -- and none on the polls in between."""
    c, _, url = sqs_client(nat, sqs_server)
    p, _ = scaler(nat, kube_server, "scale", max_=1, min_=1)
    kube_server.set_replicas("ml", "worker", 1)
    clock = nat.VirtualClock(0)
    cfg = nat.LoopConfig()
    cfg.poll_period_ns = 5 * 10**9
    cfg.scale_up_cool_down_ns = 10 * 10**9
    cfg.scale_down_cool_down_ns = 30 * 10**9
    cfg.prefetch = True
    cfg.prewarm_ns = 200_000  # the CLI default: connections are checked (or dialled) before a poll
    r = nat.Runner(cfg, c, p, clock, capture_logger([]))
    r.arm()
    sqs_server.set_attributes(url, {n: "0" for n in NAMES})
    gets0 = kube_server.gets()
    recs = r.steps(60)
    assert [i + 1 for i, x in enumerate(recs) if x["down"] == "noop"] == list(range(6, 61, 6))
    assert [i + 1 for i, x in enumerate(recs) if x["prefetched"]] == list(range(6, 61, 6))
    assert kube_server.gets() - gets0 == 10 and all(x["prefetch_used"] for x in recs if x["prefetched"])


def test_adaptive_busy_poll_tracks_peer_rtt(nat, kube_server):
    c = nat.HttpClient(kube_server.url)
    c.set_busy_poll(25_000)
    kube_server.set_latency(3_000_000)  # a "remote" peer: spinning would only burn CPU
    for _ in range(4):
        c.request("GET", "/healthz", [("Authorization", f"Bearer {TOKEN}")])
    assert c.rtt_ewma() > 4 * 25_000  # -> spin window 0
    kube_server.set_latency(0)
    # fast local peer again -> spinning re-enabled; under a loaded test runner single round trips
    # can take >100 us, so allow the EWMA a bounded number of requests to come back down
    for _ in range(500):
        c.request("GET", "/healthz", [("Authorization", f"Bearer {TOKEN}")])
        if c.rtt_ewma() < 4 * 25_000:
            break
    assert c.rtt_ewma() < 4 * 25_000


def test_tls_reconnect_resumes_session(nat):
    """After the peer closes an idle keep-alive connection, the reconnect resumes the TLS
    session (abbreviated handshake) instead of a full one."""
    import time

    k = nat.FakeKubeServer()
    k.start("127.0.0.1", 0, True)
    try:
        t = nat.TlsOptions()
        t.ca_pem = k.cert_pem
        c = nat.HttpClient(k.url, t)
        for _ in range(4):
            assert c.request("GET", "/x")[0] == 404
            k.drop_connections()
            time.sleep(0.02)
        st = c.stats()
        assert st["connects"] == 4 and st["tls_resumptions"] == 3
        # TLS 1.3 with crypto/tls's suite order (AES-128-GCM first), as the reference's clients
        assert (st["tls_version"], st["tls_cipher"]) == ("TLSv1.3", "TLS_AES_128_GCM_SHA256")
    finally:
        k.stop()


@pytest.mark.parametrize("status,header,extra_s", [(503, "2", 2), (429, "1", 1), (503, "", 0), (502, "5", 0),
                                                     (503, "Fri, 31 Dec 1999 23:59:59 GMT", 0)])
def test_sqs_throttle_honours_retry_after(nat, sqs_server, status, header, extra_s):
    """aws-sdk-go v1.35 DefaultRetryer.RetryRules: a throttle answered 429 or 503 with an
    integer Retry-After waits that many seconds on top of the back-off (getRetryAfterDelay);
    other throttles (502) and non-integer values use the back-off alone."""
    clock = nat.VirtualClock()
    o = nat.SqsHttpOptions()
    o.region, o.endpoint = REGION, sqs_server.url
    o.min_retry_delay_ns = o.min_throttle_delay_ns = 1_000_000  # 1 ms: jitter in [1, 2) ms
    api = nat.HttpSqsApi(o, static_provider(AKID, SECRET), clock)
    url = f"{sqs_server.url}/123456789012/q"
    sqs_server.set_attributes(url, ATTRS)
    sqs_server.inject(1, nat.InjectedFault(status, "busy", retry_after=header))
    t0 = clock.now()
    assert nat.SqsClient(api, url, list(ATTRS)).num_messages() == sum(int(v) for v in ATTRS.values())
    waited = clock.now() - t0
    assert extra_s * 10**9 + 1_000_000 <= waited < extra_s * 10**9 + 2_000_000
    assert api.stats()["throttle_retries"] == 1


@pytest.mark.parametrize("mode", ["scale", "patch"])
def test_scale_subresource_forbidden_falls_back_to_deployment(nat, kube_server, mode):
    kube_server.set_rbac(["deployments:get", "deployments:update"])
    lines = []
    p, api = scaler(nat, kube_server, mode, lines=lines)
    assert p.prefetch()  # the pipelined /scale GET is refused too
    span = p.scale_up()
    assert span.wrote and kube_server.replicas("ml", "worker") == 4
    assert str(api.mode) == "ScaleMode.Deployment" and api.stats()["scale_fallbacks"] == 1
    p.scale_up()
    assert kube_server.replicas("ml", "worker") == 5 and api.stats()["scale_fallbacks"] == 1
    assert kube_server.last_path().endswith("/deployments/worker") and kube_server.last_method() == "PUT"


def test_scale_write_forbidden_writes_through_the_deployment(nat, kube_server):
    """GET on deployments/scale allowed, update not: the write goes through the Deployment when
    it is still the object that was read (same resourceVersion)."""
    kube_server.set_rbac(["deployments:get", "deployments:update", "deployments/scale:get"])
    p, api = scaler(nat, kube_server, "scale")
    span = p.scale_up()
    assert span.wrote and kube_server.replicas("ml", "worker") == 4 and kube_server.forbidden() == 1
    assert api.stats()["scale_fallbacks"] == 1


def test_missing_deployment_keeps_scale_mode(nat, kube_server):
    """A 404 from /scale because the Deployment does not exist is an error, not a fallback."""
    api = new_deployment_api(RestConfig(host=kube_server.url, bearer_token=TOKEN), "ml", "scale")
    p = nat.PodAutoScaler(api, "ghost", "ml", 5, 1, 1, 1, capture_logger([]), nat.RealClock())
    with pytest.raises(nat.NativeError, match='deployments.apps "ghost" not found'):
        p.scale_up()
    assert str(api.mode) == "ScaleMode.Scale" and api.stats()["scale_fallbacks"] == 0


def test_fallback_can_be_disabled(nat, kube_server):
    kube_server.set_rbac(["deployments:get", "deployments:update"])
    api = new_deployment_api(RestConfig(host=kube_server.url, bearer_token=TOKEN), "ml", "scale", rbac_fallback=False)
    p = nat.PodAutoScaler(api, "worker", "ml", 5, 1, 1, 1, capture_logger([]), nat.RealClock())
    with pytest.raises(nat.NativeError, match='cannot get resource "deployments/scale"'):
        p.scale_up()


def test_missing_scale_route_falls_back(nat, kube_server):
    """A 404 that names no object (no /scale route on this apiserver) switches to the
    Deployment once the Deployment itself reads fine."""
    p, api = scaler(nat, kube_server, "scale")
    kube_server.inject(1, nat.InjectedFault(404, "404 page not found"))
    assert p.scale_up().wrote and kube_server.replicas("ml", "worker") == 4
    assert api.stats()["scale_fallbacks"] == 1


def test_retry_after_wait_counts_as_liveness_progress(nat, sqs_server, kube_server):
    """a worker waiting out an apiserver Retry-After (up to an hour) is backing off
    correctly, not wedged -- /healthz must not get it restarted. Runner.idle_ns() stays ~0 for
    the whole wait."""
    import threading
    import time

    c, _, url = sqs_client(nat, sqs_server)
    p, _ = scaler(nat, kube_server, "scale")
    cfg = nat.LoopConfig()
    cfg.poll_period_ns = cfg.scale_up_cool_down_ns = cfg.scale_down_cool_down_ns = 0
    r = nat.Runner(cfg, c, p, nat.RealClock(), capture_logger([]))
    r.arm()
    sqs_server.set_attributes(url, {n: "100" for n in NAMES})
    kube_server.inject(1, nat.InjectedFault(429, "", retry_after="3600"))
    out = []
    th = threading.Thread(target=lambda: out.append(r.poll_once()))
    th.start()
    try:
        time.sleep(0.5)
        assert th.is_alive() and r.idle_ns() < 100_000_000  # in the 1 h wait, counted as progress
    finally:
        r.cancel()
        th.join(10)
    assert not th.is_alive() and out[0]["up"] == "failed"


def test_explicit_content_length_header_keeps_framing(nat):
    """A request that carries its own Content-Length is sent with that header once and the body
    right after it, so the keep-alive connection stays in sync for the next request."""
    import json

    k = nat.FakeKubeServer()
    k.require_token(TOKEN)
    k.start()
    try:
        k.add_deployment("ml", "w", 2)
        c = nat.HttpClient(k.url)
        auth = [("Authorization", f"Bearer {TOKEN}")]
        path = "/apis/apps/v1/namespaces/ml/deployments/w/scale"
        status, _, body = c.request("GET", path, auth)
        assert status == 200
        obj = json.loads(body)
        obj["spec"]["replicas"] = 5
        payload = json.dumps(obj).encode()
        status, _, _ = c.request("PUT", path, auth + [("Content-Type", "application/json"),
                                                     ("Content-Length", str(len(payload)))], payload)
        assert status == 200
        status, _, body = c.request("GET", path, auth)  # same connection: still framed correctly
        assert status == 200 and json.loads(body)["spec"]["replicas"] == 5
        assert c.stats()["connects"] == 1 and k.replicas("ml", "w") == 5
    finally:
        k.stop()


def _raw_exchange(url, data):
    import socket
    import urllib.parse

    u = urllib.parse.urlsplit(url)
    with socket.create_connection((u.hostname, u.port), timeout=10) as s:
        s.sendall(data)
        out = b""
        while True:
            chunk = s.recv(65536)
            if not chunk:
                return out
            out += chunk


def test_server_rejects_malformed_header_line_like_net_http(nat):
    """Go's net/http server answers a header line without a colon with 400 and closes; an
    obs-fold continuation line joins the previous value (textproto.ReadMIMEHeader)."""
    k = nat.FakeKubeServer()
    k.start()
    try:
        bad = _raw_exchange(k.url, b"GET /healthz HTTP/1.1\r\nHost: x\r\nno colon here\r\n\r\n")
        assert bad.startswith(b"HTTP/1.1 400 ") and b"malformed MIME header line: no colon here" in bad
        folded = _raw_exchange(k.url, b"GET /apis/apps/v1/namespaces/ml/deployments/none/scale HTTP/1.1\r\n"
                                      b"Host: x\r\nX-Long: a\r\n b\r\nConnection: close\r\n\r\n")
        assert folded.startswith(b"HTTP/1.1 404 ")
    finally:
        k.stop()


def test_client_rejects_malformed_response_header_line(nat):
    """The client reads response headers as Go's transport does: a line without a colon is
    "net/http: malformed MIME header line", an obs-fold line continues the previous value."""
    import socket
    import threading

    replies = [b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\nX-Folded: a\r\n  b\r\n\r\nok",
               b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\nbogus\r\n\r\nok"]
    ls = socket.socket()
    ls.bind(("127.0.0.1", 0))
    ls.listen(4)
    port = ls.getsockname()[1]

    def serve():
        for r in replies:
            c, _ = ls.accept()
            c.recv(65536)
            c.sendall(r)
            c.close()

    t = threading.Thread(target=serve, daemon=True)
    t.start()
    try:
        c = nat.HttpClient(f"http://127.0.0.1:{port}")
        status, headers, body = c.request("GET", "/")
        assert status == 200 and body == b"ok" and ("X-Folded", "a b") in list(headers)
        c2 = nat.HttpClient(f"http://127.0.0.1:{port}")
        with pytest.raises(nat.NativeError, match="malformed MIME header line: bogus"):
            c2.request("GET", "/")
    finally:
        t.join(timeout=10)
        ls.close()


def test_signature_reused_only_within_its_second_and_credentials(nat, sqs_server):
    """The prepared SQS request's signed headers are reused while X-Amz-Date (one-second
    resolution) and the credentials are unchanged -- the same bytes a fresh signature gives --
    and re-signed at the next second or after a credential rotation."""
    token = ["t1"]

    class Rotating(nat.CredentialsProvider):
        def retrieve(self):  # expired at once: fetched again for every call
            return nat.Credentials(AKID, SECRET, token[0], 1, "Rotating")

    clock = nat.VirtualClock()  # starts on a whole second of unix time
    api = new_sqs_api(REGION, clock, endpoint=sqs_server.url, credentials=Rotating())
    url = f"{sqs_server.url}/123456789012/jobs"
    c = nat.SqsClient(api, url, NAMES)
    sqs_server.set_attributes(url, ATTRS)
    seen = []
    for i, step_ms in enumerate((0, 400, 599, 1, 0)):
        clock.advance(step_ms * 1_000_000)
        if i == 4:
            token[0] = "t2"
        assert c.num_messages() == 18
        h = dict(sqs_server.last_headers())
        seen.append((h["X-Amz-Date"], h["Authorization"], h.get("X-Amz-Security-Token")))
    assert sqs_server.signature_failures() == 0
    assert seen[0] == seen[1] == seen[2]  # same second, same credentials
    assert seen[3][0] != seen[2][0] and seen[3][1] != seen[2][1]  # next second: signed again
    assert seen[4][0] == seen[3][0] and seen[4][2] == "t2" and seen[4][1] != seen[3][1]  # rotated token


def test_webhook_denial_is_not_retried_through_the_deployment(nat, kube_server):
    """A 403 from an admission webhook (Gatekeeper, Kyverno) judged the write itself: the /scale
    -> Deployment fallback is for RBAC refusing the subresource only, or the same write would
    step around a policy that matches deployments/scale."""
    import json

    lines = []
    p, api = scaler(nat, kube_server, "scale", lines=lines)
    status = {"kind": "Status", "apiVersion": "v1", "status": "Failure", "reason": "Forbidden", "code": 403,
              "message": 'admission webhook "validate.kyverno.svc-fail" denied the request: resource Deployment/ml/worker '
                         'was blocked: replicas must stay under policy'}
    kube_server.inject(1, nat.InjectedFault(403, json.dumps(status), "application/json", method="PUT"))
    with pytest.raises(nat.NativeError, match="admission webhook"):
        p.scale_up()
    assert kube_server.replicas("ml", "worker") == 3  # nothing was written through the Deployment
    assert str(api.mode) == "ScaleMode.Scale" and api.stats()["scale_fallbacks"] == 0
    assert not any("not usable" in l for l in lines)
    assert kube_server.last_method() == "PUT" and kube_server.last_path().endswith("/scale")
    assert p.scale_up().wrote and kube_server.replicas("ml", "worker") == 4  # still /scale afterwards


def test_pipelined_get_never_dials_inside_the_sqs_call(nat, sqs_server):
    """An apiserver that accepts TCP but never completes the TLS handshake: the pipelined GET is
    not sent from inside the SQS call (it would dial on the SQS call's deadline), so the depth
    read succeeds at once; the synchronous GET then times out on its own deadline."""
    import socket
    import time

    tarpit = socket.socket()
    tarpit.bind(("127.0.0.1", 0))
    tarpit.listen(8)
    try:
        host = f"https://127.0.0.1:{tarpit.getsockname()[1]}"
        api = new_deployment_api(RestConfig(host=host, bearer_token=TOKEN, insecure=True), "ml", "scale",
                                 timeout_ns=1_500_000_000)
        p = nat.PodAutoScaler(api, "worker", "ml", 5, 1, 1, 1, capture_logger([]), nat.RealClock())
        c, _, url = sqs_client(nat, sqs_server)
        sqs_server.set_attributes(url, {n: "100" for n in NAMES})
        cfg = nat.LoopConfig()
        cfg.poll_period_ns = 0
        cfg.scale_up_cool_down_ns = 0
        cfg.prefetch = True
        r = nat.Runner(cfg, c, p, nat.RealClock(), capture_logger([]))
        r.arm()
        t0 = time.perf_counter()
        rec = r.steps(1)[0]
        assert rec["depth"] == 300 and not rec["prefetched"]
        assert rec["depth_ns"] < 500_000_000  # the SQS call did not wait for the apiserver
        assert rec["up"] == "failed" and "timeout" in rec["error"]
        assert time.perf_counter() - t0 < 10
    finally:
        tarpit.close()


@pytest.mark.parametrize("hot", [False, True])
def test_timed_tls_server_serves_and_stops_with_an_idle_client(nat, hot):
    """A client that finished its TLS handshake and sent nothing yet (a connection dialled ahead
    by --poll-prewarm) must neither hold up the hot server's single thread nor its stop(): the
    hot loop only peeks for the receive stamp, and stop() shuts client sockets down before it
    joins the serving thread."""
    import socket
    import ssl
    import threading
    import time

    srv = nat.FakeKubeServer()
    srv.set_hot(hot)
    srv.set_timing(True)
    srv.start("127.0.0.1", 0, True)
    srv.add_deployment("ns", "d", 3)
    ctx = ssl.create_default_context()
    ctx.check_hostname = False
    ctx.verify_mode = ssl.CERT_NONE
    idle = ctx.wrap_socket(socket.create_connection(("127.0.0.1", srv.port)))  # handshake done, no request
    try:
        tls = nat.TlsOptions()
        tls.ca_pem = srv.cert_pem
        c = nat.HttpClient(srv.url, tls, 5 * nat.SECOND)
        t0 = time.monotonic()
        status, _, _ = c.request("GET", "/apis/apps/v1/namespaces/ns/deployments/d")
        assert status in (200, 401) and time.monotonic() - t0 < 2.0
        c.close()
        done = threading.Event()
        threading.Thread(target=lambda: (srv.stop(), done.set()), daemon=True).start()
        assert done.wait(10), "stop() hung on an idle client"
    finally:
        idle.close()
