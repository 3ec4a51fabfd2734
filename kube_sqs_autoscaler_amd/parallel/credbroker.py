"""The CLI's one AWS credential source per region (csrc/core/cred_slot.h).

The reference fetches credentials once per process and expiry (one session,
/root/reference/sqs/sqs.go:36); N queues each running the chain would make N STS / ECS / IMDS
calls per expiry. :class:`CredentialBroker` keeps the chain in one thread of the CLI process:
one ``SharedCredentialSlot`` per region in an anonymous shared mapping (created before
``--worker-processes`` forks its workers, so they inherit it), a thread that fills each slot a
while ahead of the queues' refresh window (up to 15 minutes) or when a queue asks (a set about to expire, or one
the service rejected), and in each queue -- worker thread or worker process -- a native
``SlotCredentialsProvider`` that reads the slot and waits (cancellably) for the next set when
its own is no longer good. No poll or warm-up runs a fetch, and a refresh that fails ahead of
time keeps the set that still signs.
"""
from __future__ import annotations

import ctypes
import mmap
import threading
from typing import Dict, Iterable, Mapping, Optional

from ..ops import native
from ..sqs.credentials import make_chain_provider

# Queues refresh their copy 5 minutes before expiry (CachedCredentials, the SDK's window). The
# broker fills the slot ahead of that, so a queue finds the next set already there: halfway
# between its fetch and the queues' window, but at least MIN_LEAD_NS and at most MAX_LEAD_NS
# early (an hour-long set: 15 minutes ahead of the window, so a credential endpoint may be down
# that long without a poll failing) -- and not more often than every MIN_REFRESH_NS on its own
# (a refresh that failed is retried that often; so is a set too short for the minimum lead).
WORKER_WINDOW_NS = 5 * 60 * 1_000_000_000
MIN_LEAD_NS = 60 * 1_000_000_000
MAX_LEAD_NS = 15 * 60 * 1_000_000_000
MIN_REFRESH_NS = 10 * 1_000_000_000


def refresh_due_at(fetched_at_ns: int, expires_ns: int) -> Optional[int]:
    """When the broker refreshes a set it fetched at ``fetched_at_ns`` (None: never, for a set
    that does not expire)."""
    if not expires_ns:
        return None
    before_window = max(0, expires_ns - fetched_at_ns - WORKER_WINDOW_NS)
    lead = min(MAX_LEAD_NS, before_window, max(MIN_LEAD_NS, before_window // 2))
    return expires_ns - WORKER_WINDOW_NS - lead


class CredentialBroker:
    def __init__(self, regions: Iterable[str], environ: Optional[Mapping[str, str]] = None, clock=None,
                 poll_s: float = 0.2, providers: Optional[Dict[str, object]] = None):
        """``providers``: the chain per region (default: the SDK chain for that region).
        ``poll_s``: how often the serving thread looks at the slots -- what a queue that asks for a
        new set waits at most on top of the fetch (5 wake-ups a second: a fraction of a
        millicore)."""
        nat = native()
        self.regions = sorted(set(regions))
        self.environ = environ
        self.clock = clock or nat.RealClock()
        self.poll_s = poll_s
        self._providers = dict(providers or {})
        size = nat.credential_slot_size()
        self._slot = (size + mmap.PAGESIZE - 1) // mmap.PAGESIZE * mmap.PAGESIZE
        self._mm = mmap.mmap(-1, max(1, len(self.regions)) * self._slot, flags=mmap.MAP_SHARED | mmap.MAP_ANONYMOUS)
        self._buf = ctypes.c_char.from_buffer(self._mm)
        base = ctypes.addressof(self._buf)
        self.addrs = {r: base + i * self._slot for i, r in enumerate(self.regions)}
        for a in self.addrs.values():
            nat.init_credential_slot(a)
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._last_fetch: Dict[str, int] = {}
        self._due_at: Dict[str, Optional[int]] = {}  # when each region's set is refreshed ahead of time
        self.fetches = 0
        self.fetches_by_region: Dict[str, int] = {r: 0 for r in self.regions}
        self.refresh_errors = 0  # failed refreshes ahead of time (the set in the slot kept)

    def provider_for(self, region: str, clock=None):
        """A queue's credential source for ``region`` (a worker process calls it after the fork)."""
        return native().SlotCredentialsProvider(self.addrs[region], clock or native().RealClock(), WORKER_WINDOW_NS)

    def _chain(self, region: str):
        p = self._providers.get(region)
        if p is None:
            p = self._providers[region] = make_chain_provider(environ=self.environ, region=region)
        return p

    def serve_once(self) -> int:
        """Fills every slot that needs it; returns how many were fetched."""
        nat = native()
        n = 0
        for region, addr in self.addrs.items():
            now = self.clock.unix_nanos()
            asked = nat.credential_slot_needs_fetch(addr, now, 0)  # none yet, a worker asked, expired
            due_at = self._due_at.get(region)
            due = due_at is not None and now >= due_at and now - self._last_fetch.get(region, 0) >= MIN_REFRESH_NS
            if not (asked or due):
                continue
            self._last_fetch[region] = now
            n += 1
            self.fetches += 1
            self.fetches_by_region[region] += 1
            try:
                creds = self._chain(region).retrieve()
                nat.publish_credentials(addr, creds)
                self._due_at[region] = refresh_due_at(now, creds.expires_unix_ns)
            except Exception as e:  # noqa: BLE001
                # Every worker waiting on the slot gets the error. A refresh ahead of time that
                # fails leaves the current set in place (it still signs) and is tried again.
                if asked:
                    nat.publish_credential_error(addr, str(e))
                else:
                    self.refresh_errors += 1
        return n

    def start(self) -> None:
        """The serving thread (with ``--worker-processes``, start it after the workers have forked)."""
        if self._thread is not None:
            return

        def loop():
            while not self._stop.is_set():
                self.serve_once()
                self._stop.wait(self.poll_s)

        self._thread = threading.Thread(target=loop, name="ksa-credentials", daemon=True)
        self._thread.start()

    def stop(self, timeout: float = 1.0) -> bool:
        """Stops the serving thread; False when it is still inside a fetch after ``timeout``
        (a hung credential endpoint: the thread is a daemon and ends with the process)."""
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=timeout)
            if self._thread.is_alive():
                return False
            self._thread = None
        return True

    def close(self) -> None:
        # an idle serving thread ends at once; one inside a fetch is not waited for
        if not self.stop(timeout=0.1):
            return  # the thread may still publish into the slots: leave them mapped
        del self._buf
        self._mm.close()
