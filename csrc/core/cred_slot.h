// One AWS credential set shared by the worker processes of --worker-processes.
//
// The reference builds one session per process (/root/reference/sqs/sqs.go:36): one credential
// fetch per expiry. A thread fleet shares one SharedCredentialsProvider (sigv4.h) per region; a
// process fleet forks one worker per queue, and without this each worker would run the chain
// itself -- N STS / ECS / IMDS calls per expiry. Instead the supervisor keeps the chain and
// publishes its current set into a slot of anonymous shared memory (one per region); each worker
// reads it through SlotCredentialsProvider and, when its copy nears expiry or the set was
// rejected, asks the supervisor for a newer one and waits for it.
//
// Deliberate deviation (docs/PARITY_MATRIX.md): the SDK treats its 5-minute expiry window as
// hard -- inside it, a call whose refresh fails fails. Here a refresh that fails while the set in
// the slot still signs for more than kStaleSkew leaves that set in place, marked with the
// refresh's error, and the workers keep signing with it (counted in `stale_signs`) until a
// refresh succeeds or the set reaches Expiration - kStaleSkew; only then does the chain's error
// reach a poll. A set the service rejected (ExpiredToken) is never signed with again.
//
// Like SharedWorkerState (runner.h): lock-free atomics only (address-free on x86-64), each word
// with one writer -- the supervisor for the set, its generation and its error; the workers for
// the `wanted` generation (an atomic max). The set is written under a seqlock. Nobody polls for
// the other side: a worker's ask bumps `asks` and a publication bumps `published`, each followed
// by a process-shared futex wake, so the supervisor's serving thread and the waiting workers
// sleep until there is something to read (the waits also time out, to look at cancel and stop).
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>

#include "clock.h"
#include "sigv4.h"

namespace ksa {

struct SharedCredentialSlot {
  static constexpr size_t kBytes = 12 * 1024;  // key id + secret + session token + names
  std::atomic<uint64_t> seq;         // odd while the supervisor writes the set
  std::atomic<uint64_t> generation;  // sets (or errors) published so far; 0: none yet
  std::atomic<uint64_t> wanted;      // the newest generation a worker asked to be replaced
  std::atomic<uint64_t> rejected;    // the newest generation a worker saw the service reject
  std::atomic<uint64_t> stale_signs; // SQS requests signed with a set kept after a failed refresh
  std::atomic<uint32_t> asks;       // futex word: bumped by every request_credentials()
  std::atomic<uint32_t> published;  // futex word: bumped by every publication
  std::atomic<int64_t> expires_unix_ns;
  // access key id, secret, token, provider name, error, refresh error (the set kept after a
  // failed refresh: why it was not replaced)
  std::atomic<uint32_t> len[6];
  std::atomic<uint64_t> words[kBytes / 8];
};

SharedCredentialSlot* init_credential_slot(void* at);
// Supervisor side: publish a set (error empty) or the chain's error (every waiting worker's
// fetch then fails with it); either bumps the generation. `refresh_error` non-empty: `c` is the
// set already in the slot, kept because its refresh failed with that error.
void publish_credentials(SharedCredentialSlot* s, const Credentials& c, const std::string& refresh_error = "");
void publish_credential_error(SharedCredentialSlot* s, const std::string& error);
// A consistent read: false while nothing is published (or a writer kept the seqlock busy).
bool read_credential_slot(const SharedCredentialSlot* s, Credentials* c, std::string* error, uint64_t* generation,
                          std::string* refresh_error = nullptr);
// Worker side: ask for a set newer than `generation` (an atomic max).
void request_credentials(SharedCredentialSlot* s, uint64_t generation);
// Worker side: the service rejected generation `generation`'s set -- no worker signs with it
// again -- and a newer one is asked for.
void reject_credentials(SharedCredentialSlot* s, uint64_t generation);
// Supervisor side: whether the slot needs a fetch -- nothing published, a worker asked to
// replace the current generation, or the set expires within `window` of `unix_now`.
bool credential_slot_needs_fetch(const SharedCredentialSlot* s, int64_t unix_now, int64_t window);
// Supervisor side: sleep until a worker asks (`asks` moves past `seen`), `timeout` passes or
// credential_slot_poke() is called; returns the current `asks`.
uint32_t credential_slot_wait_ask(SharedCredentialSlot* s, uint32_t seen, Nanos timeout);
uint32_t credential_slot_asks(const SharedCredentialSlot* s);
// Wakes every thread waiting on the slot (supervisor and workers): the supervisor's stop.
void credential_slot_poke(SharedCredentialSlot* s);
// Whether the slot's set may still be signed with at `unix_now`: a set (not an error) that was
// not rejected and does not expire within `skew`. The supervisor keeps such a set when its
// refresh fails.
bool credential_slot_still_signs(const SharedCredentialSlot* s, int64_t unix_now, int64_t skew);

// A worker's credential source: the slot's set while it is outside `window` of its expiry, or
// inside it while the supervisor's refresh is failing and the set signs for more than `skew`;
// otherwise a request to the supervisor and a wait (up to `wait_limit`, or until cancel()) for a
// newer generation.
class SlotCredentialsProvider final : public CredentialsProvider {
 public:
  SlotCredentialsProvider(SharedCredentialSlot* slot, std::function<int64_t()> unix_now, int64_t window,
                          Nanos wait_limit = 15 * kSecond, int64_t skew = kStaleSkew)
      : slot_(slot), now_(std::move(unix_now)), window_(window), wait_limit_(wait_limit), skew_(skew) {}
  Result<Credentials> retrieve() override;
  void stale(const Credentials& c) override;
  // The worker stops: a retrieve() waiting for the supervisor returns "request canceled" at once.
  void cancel() override;
  // Counts a request signed with a kept set into the slot (every worker of the slot, threads and
  // processes alike, adds to one count).
  void signed_with_kept(const Credentials& c) override;

 private:
  Result<Credentials> ride(Credentials c);
  std::atomic<bool> cancelled_{false};
  SharedCredentialSlot* slot_;
  std::function<int64_t()> now_;
  int64_t window_;
  Nanos wait_limit_;
  int64_t skew_;
};

}  // namespace ksa
