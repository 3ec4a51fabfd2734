"""client-go's request retries (k8s.io/client-go v0.19 rest/request.go ``request`` + ``checkWait``),
which the reference inherits for every Deployment GET and PUT (/root/reference/scale/scale.go:55,72):

* a 429 or 5xx response with an integer ``Retry-After`` is retried after that many seconds, at
  most 10 times (API Priority and Fairness and max-inflight rejections carry ``Retry-After: 1``);
* a GET whose connection was reset or hit EOF is retried as if it had ``Retry-After: 1``; writes
  are not (they are not idempotent);
* anything else (no header, an HTTP-date, 4xx) fails at once.

The waits run on the client's clock: a VirtualClock makes them instant and measurable.
"""
import pytest

from kube_sqs_autoscaler_amd.autoscaler import new_deployment_api
from kube_sqs_autoscaler_amd.kube.config import RestConfig
from kube_sqs_autoscaler_amd.utils.log import capture_logger

TOKEN = "tok-retry"
S = 1_000_000_000


@pytest.fixture
def kube(nat):
    k = nat.FakeKubeServer()
    k.require_token(TOKEN)
    k.start()
    k.add_deployment("ml", "w", 1)
    yield k
    k.stop()


def scaler(nat, kube, clock, mode="scale", max_pods=5):
    api = new_deployment_api(RestConfig(host=kube.url, bearer_token=TOKEN), "ml", mode, 5 * S, clock)
    logs = []
    return api, nat.PodAutoScaler(api, "w", "ml", max_pods, 1, 1, 1, capture_logger(logs), clock), logs


def test_retry_after_on_429_then_success(nat, kube):
    clock = nat.VirtualClock()
    api, p, _ = scaler(nat, kube, clock)
    kube.inject(2, nat.InjectedFault(429, "slow down", retry_after="1"))
    t0 = clock.now()
    p.scale_up()
    assert kube.replicas("ml", "w") == 2
    assert api.stats()["retry_after"] == 2
    assert clock.now() - t0 == 2 * S  # slept Retry-After seconds twice


@pytest.mark.parametrize("status,retry_after,retried", [
    (503, "3", True), (500, "0", True), (429, "+2", True),
    (503, "", False),  # no header
    (500, "Wed, 21 Oct 2015 07:28:00 GMT", False),  # strconv.Atoi fails: not retried
    (400, "1", False),  # only 429 and 5xx wait (a 404 on /scale may switch to the Deployment instead)
])
def test_check_wait_rules(nat, kube, status, retry_after, retried):
    clock = nat.VirtualClock()
    api, p, _ = scaler(nat, kube, clock)
    kube.inject(1, nat.InjectedFault(status, "x", retry_after=retry_after))
    if retried:
        p.scale_up()
        assert kube.replicas("ml", "w") == 2 and api.stats()["retry_after"] == 1
    else:
        with pytest.raises(nat.NativeError):
            p.scale_up()
        assert kube.replicas("ml", "w") == 1 and api.stats()["retry_after"] == 0


def test_gives_up_after_ten_retries(nat, kube):
    clock = nat.VirtualClock()
    api, p, _ = scaler(nat, kube, clock)
    kube.inject(11, nat.InjectedFault(429, "", retry_after="1"))
    with pytest.raises(nat.NativeError, match="too many requests"):
        p.scale_up()
    assert api.stats()["retry_after"] == 10
    kube.inject(10, nat.InjectedFault(429, "", retry_after="1"))
    p.scale_up()  # ten 429s then success: within the budget
    assert kube.replicas("ml", "w") == 2


def test_reset_get_is_retried_but_write_is_not(nat, kube):
    clock = nat.VirtualClock()
    api, p, _ = scaler(nat, kube, clock)
    kube.inject(1, nat.InjectedFault(0, "", "text/plain", True))  # the GET's connection closes unanswered
    t0 = clock.now()
    p.scale_up()
    assert kube.replicas("ml", "w") == 2 and api.stats()["retry_after"] == 1
    assert clock.now() - t0 == 1 * S
    # a write whose (fresh) connection closes unanswered is not replayed
    obj = api.get("w")
    api2, _, _ = scaler(nat, kube, clock)
    kube.inject(1, nat.InjectedFault(0, "", "text/plain", True))
    with pytest.raises(nat.NativeError, match="EOF|closed|reset"):
        api2.update("w", obj, 4)
    assert kube.replicas("ml", "w") == 2 and api2.stats()["retry_after"] == 0


def test_pipelined_read_falls_back_to_a_retried_get(nat, kube):
    clock = nat.VirtualClock()
    api, _, _ = scaler(nat, kube, clock)
    kube.inject(1, nat.InjectedFault(429, "", retry_after="1"))
    assert api.begin_get("w")
    obj = api.finish_get()
    assert obj.replicas == 1 and api.stats()["retry_after"] == 1


def test_written_put_on_a_reused_connection_is_never_replayed(nat, kube):
    """a PUT fully written on a reused keep-alive connection that then closes without
    a response byte must not be sent again (Go's transport replays only requests that never
    reached the wire or are idempotent; client-go never retries a write on EOF). A replay could
    apply the write twice, or 409 on its own first copy and skip the cool-down refresh."""
    clock = nat.VirtualClock()
    api, _, _ = scaler(nat, kube, clock)
    obj = api.get("w")  # the connection is now reused
    before = kube.requests()
    kube.inject(1, nat.InjectedFault(0, "", "text/plain", True))  # the PUT's connection closes unanswered
    with pytest.raises(nat.NativeError, match="EOF|closed|reset"):
        api.update("w", obj, 4)
    assert kube.requests() - before == 1  # exactly one write on the wire
    assert api.stats()["http"]["reconnect_retries"] == 0 and api.stats()["retry_after"] == 0


def test_reused_get_dropped_is_replayed_at_once(nat, kube):
    clock = nat.VirtualClock()
    api, _, _ = scaler(nat, kube, clock)
    api.get("w")
    kube.inject(1, nat.InjectedFault(0, "", "text/plain", True))
    t0 = clock.now()
    assert api.get("w").replicas == 1
    st = api.stats()
    assert st["http"]["reconnect_retries"] == 1 and st["retry_after"] == 0 and clock.now() == t0


def test_idle_closed_connection_is_redialled_before_writing(nat, kube):
    """The apiserver closed the idle keep-alive connection between polls: the next request --
    a PUT included -- goes out on a fresh connection, never into the dead one."""
    import time

    clock = nat.VirtualClock()
    api, _, _ = scaler(nat, kube, clock)
    obj = api.get("w")
    kube.drop_connections()
    # let the FIN arrive, and leave the 20 ms after a response in which a connection is reused
    # without the idle-close peek (http.cc kFreshConnNs)
    time.sleep(0.05)
    api.update("w", obj, 3)
    assert kube.replicas("ml", "w") == 3
    st = api.stats()["http"]
    assert st["idle_closed"] == 1 and st["reconnect_retries"] == 0 and st["connects"] == 2
