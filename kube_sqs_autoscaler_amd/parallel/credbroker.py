"""The CLI's one AWS credential source per region (csrc/core/cred_slot.h).

The reference fetches credentials once per process and expiry (one session,
/root/reference/sqs/sqs.go:36); N queues each running the chain would make N STS / ECS / IMDS
calls per expiry. :class:`CredentialBroker` keeps the chain in the CLI process: one
``SharedCredentialSlot`` per region in an anonymous shared mapping (created before
``--worker-processes`` forks its workers, so they inherit it), one serving thread per region that
fills its slot a while ahead of the queues' refresh window (up to 15 minutes) or when a queue asks
(a set about to expire, or one the service rejected), and in each queue -- worker thread or
worker process -- a native ``SlotCredentialsProvider`` that reads the slot and waits (cancellably)
for the next set when its own is no longer good. No poll or warm-up runs a fetch.

Each region has its own thread because a fetch can block for seconds (STS 10 s, ECS 5 s,
``credential_process`` 60 s: sqs/credentials.py) and the queues of one region must not wait out
another region's hung endpoint (/root/reference/sqs/sqs.go:35-43: the client per queue's region).

A refresh that fails while the set in the slot still signs for more than a minute keeps that
set, marked with the error: the queues go on signing with it past the SDK's 5-minute window
(``ksa_aws_credential_stale_signs_total``, one warning per set) until a refresh succeeds or the
set is a minute from its Expiration; only then does the chain's error reach a poll. A deliberate
deviation from aws-sdk-go, whose window is hard (docs/PARITY_MATRIX.md): a poll signed with a
key that is still valid decides what the reference decides on a successful read.
"""
from __future__ import annotations

import ctypes
import mmap
import threading
import time
from datetime import datetime, timezone
from typing import Callable, Dict, Iterable, Mapping, Optional

from ..ops import native
from ..sqs.credentials import make_chain_provider

# Queues refresh their copy 5 minutes before expiry (CachedCredentials, the SDK's window). The
# broker fills the slot ahead of that, so a queue finds the next set already there: halfway
# between its fetch and the queues' window, but at least MIN_LEAD_NS and at most MAX_LEAD_NS
# early (an hour-long set: 15 minutes ahead of the window) -- and not more often than every
# MIN_REFRESH_NS on its own (a refresh that failed is retried that often; so is a set too short
# for the minimum lead). A set whose refresh keeps failing is signed with until STALE_SKEW_NS
# before it expires.
WORKER_WINDOW_NS = 5 * 60 * 1_000_000_000
MIN_LEAD_NS = 60 * 1_000_000_000
MAX_LEAD_NS = 15 * 60 * 1_000_000_000
MIN_REFRESH_NS = 10 * 1_000_000_000
STALE_SKEW_NS = 60 * 1_000_000_000


def refresh_due_at(fetched_at_ns: int, expires_ns: int) -> Optional[int]:
    """When the broker refreshes a set it fetched at ``fetched_at_ns`` (None: never, for a set
    that does not expire)."""
    if not expires_ns:
        return None
    before_window = max(0, expires_ns - fetched_at_ns - WORKER_WINDOW_NS)
    lead = min(MAX_LEAD_NS, before_window, max(MIN_LEAD_NS, before_window // 2))
    return expires_ns - WORKER_WINDOW_NS - lead


def _utc(ns: int) -> str:
    return datetime.fromtimestamp(ns / 1e9, timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


class CredentialBroker:
    def __init__(self, regions: Iterable[str], environ: Optional[Mapping[str, str]] = None, clock=None,
                 poll_s: float = 0.2, providers: Optional[Dict[str, object]] = None,
                 log: Optional[Callable[[str, str], None]] = None):
        """``providers``: the chain per region (default: the SDK chain for that region).
        ``poll_s``: how often each region's serving thread looks at its slot for a refresh that
        is due (5 wake-ups a second per region: a fraction of a millicore); a queue that asks for
        a new set wakes it at once (a futex on the slot). ``log(level, message)``: where the
        warnings go."""
        nat = native()
        self.regions = sorted(set(regions))
        self.environ = environ
        self.clock = clock or nat.RealClock()
        self.poll_s = poll_s
        self.log = log
        self._providers = dict(providers or {})
        self.skew_ns = nat.CREDENTIAL_STALE_SKEW_NS
        assert self.skew_ns == STALE_SKEW_NS
        size = nat.credential_slot_size()
        self._slot = (size + mmap.PAGESIZE - 1) // mmap.PAGESIZE * mmap.PAGESIZE
        self._mm = mmap.mmap(-1, max(1, len(self.regions)) * self._slot, flags=mmap.MAP_SHARED | mmap.MAP_ANONYMOUS)
        self._buf = ctypes.c_char.from_buffer(self._mm)
        base = ctypes.addressof(self._buf)
        self.addrs = {r: base + i * self._slot for i, r in enumerate(self.regions)}
        for a in self.addrs.values():
            nat.init_credential_slot(a)
        self._stop = threading.Event()
        self._closed = False  # the slots unmapped (close())
        self._threads: Dict[str, threading.Thread] = {}
        self._lock = threading.Lock()  # the counters below (one serving thread per region)
        self._last_fetch: Dict[str, int] = {}
        self._due_at: Dict[str, Optional[int]] = {}  # when each region's set is refreshed ahead of time
        self._warned: Dict[str, tuple] = {}  # the kept set each region last warned about
        self.fetches = 0
        self.fetches_by_region: Dict[str, int] = {r: 0 for r in self.regions}
        self.refresh_errors = 0  # failed fetches that left a set still signing in the slot

    def provider_for(self, region: str, clock=None):
        """A queue's credential source for ``region`` (a worker process calls it after the fork)."""
        return native().SlotCredentialsProvider(self.addrs[region], clock or native().RealClock(), WORKER_WINDOW_NS)

    def stale_signs_by_region(self) -> Dict[str, int]:
        """Per region, the signatures the queues (threads and worker processes alike: the count
        lives in the shared slot) made with a set kept after its refresh failed."""
        nat = native()
        return {r: nat.credential_slot_info(a)["stale_signs"] for r, a in self.addrs.items()}

    def _chain(self, region: str):
        with self._lock:
            p = self._providers.get(region)
            if p is None:
                p = self._providers[region] = make_chain_provider(environ=self.environ, region=region)
            return p

    def serve_region(self, region: str) -> bool:
        """Fills ``region``'s slot if it needs it; True when a fetch was made."""
        nat = native()
        addr = self.addrs[region]
        now = self.clock.unix_nanos()
        asked = nat.credential_slot_needs_fetch(addr, now, 0)  # none yet, a worker asked, expired
        due_at = self._due_at.get(region)
        due = due_at is not None and now >= due_at and now - self._last_fetch.get(region, 0) >= MIN_REFRESH_NS
        if not (asked or due):
            return False
        self._last_fetch[region] = now
        with self._lock:
            self.fetches += 1
            self.fetches_by_region[region] += 1
        try:
            creds = self._chain(region).retrieve()
        except Exception as e:  # noqa: BLE001
            self._failed(region, addr, asked, str(e))
            return True
        nat.publish_credentials(addr, creds)
        self._due_at[region] = refresh_due_at(now, creds.expires_unix_ns)
        return True

    def _failed(self, region: str, addr: int, asked: bool, error: str) -> None:
        """A fetch failed. A set that still signs (not rejected, more than STALE_SKEW_NS from
        expiry) is kept and republished with the error, so the queues sign with it instead of
        waiting; the refresh is retried every MIN_REFRESH_NS. Otherwise a queue that asked gets
        the error (as the SDK fails a call whose refresh fails), and one that did not ask keeps
        what it has."""
        nat = native()
        now = self.clock.unix_nanos()
        if nat.credential_slot_still_signs(addr, now, self.skew_ns):
            creds = nat.read_credential_slot(addr)[0]
            nat.publish_credentials(addr, creds, error)
            with self._lock:
                self.refresh_errors += 1
            key = (creds.access_key_id, creds.session_token, creds.expires_unix_ns)
            if self.log is not None and self._warned.get(region) != key:
                self._warned[region] = key
                until = (f"until {_utc(creds.expires_unix_ns - self.skew_ns)} (a minute before it expires) or "
                         if creds.expires_unix_ns else "")
                self.log("warning", f"AWS credential refresh for {region} failed: {error}; the queues keep signing "
                                    f"with the current set from {creds.provider_name or 'the chain'} {until}"
                                    "until a refresh succeeds")
        elif asked:
            nat.publish_credential_error(addr, error)

    def serve_once(self) -> int:
        """Fills every slot that needs it, one region after the other; returns how many were
        fetched (the serving threads call serve_region concurrently)."""
        return sum(self.serve_region(r) for r in self.regions)

    def start(self) -> None:
        """One serving thread per region (with ``--worker-processes``, start them after the
        workers have forked)."""
        if self._threads:
            return

        nat = native()
        timeout_ns = int(self.poll_s * 1e9)

        def loop(region: str):
            addr = self.addrs[region]
            while not self._stop.is_set():
                seen = nat.credential_slot_asks(addr)  # an ask during the serve below: serve again
                try:
                    self.serve_region(region)
                except Exception as e:  # noqa: BLE001 -- a broken slot must not end the thread
                    if self.log is not None:
                        self.log("error", f"AWS credential broker ({region}): {type(e).__name__}: {e}")
                if not self._stop.is_set():
                    nat.credential_slot_wait_ask(addr, seen, timeout_ns)

        for region in self.regions:
            t = threading.Thread(target=loop, args=(region,), name=f"ksa-credentials-{region}", daemon=True)
            self._threads[region] = t
            t.start()

    def stop(self, timeout: float = 1.0) -> bool:
        """Stops the serving threads; False when one is still inside a fetch after ``timeout``
        (a hung credential endpoint: the threads are daemons and end with the process)."""
        self._stop.set()
        if self._threads and not self._closed:  # wake the threads sleeping between looks
            for addr in self.addrs.values():
                native().credential_slot_poke(addr)
        deadline = time.monotonic() + timeout
        for t in self._threads.values():
            t.join(timeout=max(0.0, deadline - time.monotonic()))
        if any(t.is_alive() for t in self._threads.values()):
            return False
        self._threads = {}
        return True

    def close(self) -> None:
        # idle serving threads end at once; one inside a fetch is not waited for
        if self._closed or not self.stop(timeout=0.1):
            return  # (a thread may still publish into the slots: leave them mapped)
        self._closed = True
        del self._buf
        self._mm.close()
