#include "cred_slot.h"

#include <linux/futex.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <climits>

#include <algorithm>
#include <cstring>
#include <new>

namespace ksa {

namespace {

enum Part : int { kAkid = 0, kSecret = 1, kToken = 2, kName = 3, kError = 4, kRefreshError = 5, kParts = 6 };

void nap(Nanos ns) {
  struct timespec ts = {static_cast<time_t>(ns / kSecond), static_cast<long>(ns % kSecond)};
  nanosleep(&ts, nullptr);
}

// Process-shared futex on a 32-bit atomic of the slot (the mapping is MAP_SHARED, so no
// FUTEX_PRIVATE_FLAG). std::atomic<uint32_t> is the plain word on Linux.
static_assert(sizeof(std::atomic<uint32_t>) == sizeof(uint32_t), "futex word");

constexpr Nanos kCancelCheck = 20 * kMillisecond;

void futex_wait(std::atomic<uint32_t>* word, uint32_t seen, Nanos timeout) {
  if (timeout <= 0) return;
  struct timespec ts = {static_cast<time_t>(timeout / kSecond), static_cast<long>(timeout % kSecond)};
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(word), FUTEX_WAIT, seen, &ts, nullptr, 0);
}

void futex_wake_all(std::atomic<uint32_t>* word) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(word), FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0);
}

void publish_parts(SharedCredentialSlot* s, const std::string (&parts)[kParts], int64_t expires) {
  size_t total = 0;
  for (const auto& p : parts) total += p.size();
  if (total > SharedCredentialSlot::kBytes) {
    std::string err[kParts];
    err[kError] = "credentials do not fit the worker processes' shared slot (" + std::to_string(total) + " bytes)";
    publish_parts(s, err, 0);
    return;
  }
  std::string all;
  all.reserve(total);
  for (const auto& p : parts) all += p;
  const uint64_t seq = s->seq.load(std::memory_order_relaxed);
  s->seq.store(seq + 1, std::memory_order_relaxed);  // odd: being written
  std::atomic_thread_fence(std::memory_order_release);
  for (size_t w = 0; w * 8 < all.size(); ++w) {
    uint64_t word = 0;
    std::memcpy(&word, all.data() + w * 8, std::min<size_t>(8, all.size() - w * 8));
    s->words[w].store(word, std::memory_order_relaxed);
  }
  for (int i = 0; i < kParts; ++i) s->len[i].store(static_cast<uint32_t>(parts[i].size()), std::memory_order_relaxed);
  s->expires_unix_ns.store(expires, std::memory_order_relaxed);
  s->seq.store(seq + 2, std::memory_order_release);
  s->generation.fetch_add(1, std::memory_order_acq_rel);
  s->published.fetch_add(1, std::memory_order_release);
  futex_wake_all(&s->published);
}

}  // namespace

SharedCredentialSlot* init_credential_slot(void* at) {
  auto* s = new (at) SharedCredentialSlot;
  s->seq.store(0, std::memory_order_relaxed);
  s->generation.store(0, std::memory_order_relaxed);
  s->wanted.store(0, std::memory_order_relaxed);
  s->rejected.store(0, std::memory_order_relaxed);
  s->stale_signs.store(0, std::memory_order_relaxed);
  s->asks.store(0, std::memory_order_relaxed);
  s->published.store(0, std::memory_order_relaxed);
  s->expires_unix_ns.store(0, std::memory_order_relaxed);
  for (auto& l : s->len) l.store(0, std::memory_order_relaxed);
  for (auto& w : s->words) w.store(0, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  return s;
}

void publish_credentials(SharedCredentialSlot* s, const Credentials& c, const std::string& refresh_error) {
  const std::string parts[kParts] = {c.access_key_id, c.secret_access_key, c.session_token, c.provider_name, "",
                                     refresh_error};
  publish_parts(s, parts, c.expires_unix_ns);
}

void publish_credential_error(SharedCredentialSlot* s, const std::string& error) {
  std::string parts[kParts];
  parts[kError] = error.empty() ? "credential fetch failed" : error;
  publish_parts(s, parts, 0);
}

bool read_credential_slot(const SharedCredentialSlot* s, Credentials* c, std::string* error, uint64_t* generation,
                          std::string* refresh_error) {
  for (int attempt = 0; attempt < 4096; ++attempt) {
    const uint64_t gen = s->generation.load(std::memory_order_acquire);
    const uint64_t before = s->seq.load(std::memory_order_acquire);
    if (gen == 0) return false;
    if (before & 1) {
      if (attempt > 64) nap(10 * kMicrosecond);
      continue;
    }
    uint32_t len[kParts];
    size_t total = 0;
    for (int i = 0; i < kParts; ++i) {
      len[i] = std::min<uint32_t>(s->len[i].load(std::memory_order_relaxed), SharedCredentialSlot::kBytes);
      total += len[i];
    }
    if (total > SharedCredentialSlot::kBytes) continue;  // torn lengths: the check below retries
    std::string all(total, '\0');
    for (size_t w = 0; w * 8 < total; ++w) {
      const uint64_t word = s->words[w].load(std::memory_order_relaxed);
      std::memcpy(&all[w * 8], &word, std::min<size_t>(8, total - w * 8));
    }
    const int64_t expires = s->expires_unix_ns.load(std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_acquire);
    if (s->seq.load(std::memory_order_relaxed) != before || s->generation.load(std::memory_order_relaxed) != gen)
      continue;
    size_t off = 0;
    std::string parts[kParts];
    for (int i = 0; i < kParts; ++i) {
      parts[i] = all.substr(off, len[i]);
      off += len[i];
    }
    *c = Credentials();
    c->access_key_id = parts[kAkid];
    c->secret_access_key = parts[kSecret];
    c->session_token = parts[kToken];
    c->provider_name = parts[kName];
    c->expires_unix_ns = expires;
    *error = parts[kError];
    if (refresh_error) *refresh_error = parts[kRefreshError];
    *generation = gen;
    return true;
  }
  return false;
}

void request_credentials(SharedCredentialSlot* s, uint64_t generation) {
  uint64_t cur = s->wanted.load(std::memory_order_relaxed);
  while (cur < generation &&
         !s->wanted.compare_exchange_weak(cur, generation, std::memory_order_acq_rel, std::memory_order_relaxed)) {
  }
  s->asks.fetch_add(1, std::memory_order_release);
  futex_wake_all(&s->asks);
}

uint32_t credential_slot_asks(const SharedCredentialSlot* s) { return s->asks.load(std::memory_order_acquire); }

uint32_t credential_slot_wait_ask(SharedCredentialSlot* s, uint32_t seen, Nanos timeout) {
  if (s->asks.load(std::memory_order_acquire) == seen) futex_wait(&s->asks, seen, timeout);
  return s->asks.load(std::memory_order_acquire);
}

void credential_slot_poke(SharedCredentialSlot* s) {
  s->asks.fetch_add(1, std::memory_order_release);
  s->published.fetch_add(1, std::memory_order_release);
  futex_wake_all(&s->asks);
  futex_wake_all(&s->published);
}

void reject_credentials(SharedCredentialSlot* s, uint64_t generation) {
  uint64_t cur = s->rejected.load(std::memory_order_relaxed);
  while (cur < generation &&
         !s->rejected.compare_exchange_weak(cur, generation, std::memory_order_acq_rel, std::memory_order_relaxed)) {
  }
  request_credentials(s, generation);
}

bool credential_slot_needs_fetch(const SharedCredentialSlot* s, int64_t unix_now, int64_t window) {
  const uint64_t gen = s->generation.load(std::memory_order_acquire);
  if (gen == 0 || s->wanted.load(std::memory_order_acquire) >= gen) return true;
  if (s->len[kError].load(std::memory_order_relaxed) > 0) return false;  // retried when a worker asks
  const int64_t expires = s->expires_unix_ns.load(std::memory_order_relaxed);
  return expires != 0 && unix_now + window >= expires;
}

bool credential_slot_still_signs(const SharedCredentialSlot* s, int64_t unix_now, int64_t skew) {
  Credentials c;
  std::string error;
  uint64_t gen = 0;
  if (!read_credential_slot(s, &c, &error, &gen) || !error.empty() || !c.valid()) return false;
  if (s->rejected.load(std::memory_order_acquire) >= gen) return false;
  return c.expires_unix_ns == 0 || unix_now + skew < c.expires_unix_ns;
}

Result<Credentials> SlotCredentialsProvider::ride(Credentials c) {
  c.kept_after_failed_refresh = true;  // the request it signs is counted (signed_with_kept)
  return Result<Credentials>::Ok(c);
}

void SlotCredentialsProvider::signed_with_kept(const Credentials& c) {
  (void)c;
  slot_->stale_signs.fetch_add(1, std::memory_order_relaxed);
}

Result<Credentials> SlotCredentialsProvider::retrieve() {
  Credentials c;
  std::string error, refresh_error;
  uint64_t gen = 0;
  const bool have = read_credential_slot(slot_, &c, &error, &gen, &refresh_error);
  // a set, not an error, that no worker saw the service reject (stale() marks the generation)
  const bool good = have && error.empty() && c.valid() && slot_->rejected.load(std::memory_order_acquire) < gen;
  int64_t now = now_();
  if (good && (c.expires_unix_ns == 0 || now + window_ < c.expires_unix_ns)) return Result<Credentials>::Ok(c);
  // Inside the window, but the supervisor's refresh failed and kept this set, which signs for a
  // while yet: sign with it (the supervisor keeps retrying on its own) rather than wait and fail.
  if (good && !refresh_error.empty() && now + skew_ < c.expires_unix_ns) return ride(c);
  // Nothing yet, an error, a rejected set, or one about to expire: ask the supervisor for the next.
  request_credentials(slot_, have ? gen : 0);
  const int64_t deadline = mono_ns() + wait_limit_;
  // Sleep on the slot's `published` word until the supervisor publishes (the ask above woke its
  // serving thread); the wait times out every kCancelCheck to look at cancel() and the deadline.
  for (;;) {
    const uint32_t seen = slot_->published.load(std::memory_order_acquire);
    if (cancelled_.load(std::memory_order_acquire)) return Result<Credentials>::Err(Status::Err("request canceled"));
    Credentials next;
    std::string next_error, next_refresh_error;
    uint64_t next_gen = 0;
    if (read_credential_slot(slot_, &next, &next_error, &next_gen, &next_refresh_error) && next_gen > gen) {
      if (!next_error.empty()) return Result<Credentials>::Err(Status::Err(next_error));
      if (next_refresh_error.empty()) return Result<Credentials>::Ok(next);
      // the refresh this worker asked for failed and the set was kept: it signs until the skew
      now = now_();
      if (slot_->rejected.load(std::memory_order_acquire) < next_gen &&
          (next.expires_unix_ns == 0 || now + skew_ < next.expires_unix_ns))
        return ride(next);
      return Result<Credentials>::Err(Status::Err(next_refresh_error));
    }
    const int64_t left = deadline - mono_ns();
    if (left <= 0) break;
    futex_wait(&slot_->published, seen, std::min<Nanos>(left, kCancelCheck));
  }
  // No answer: a set that has not expired yet still signs.
  if (good && (c.expires_unix_ns == 0 || now_() < c.expires_unix_ns)) return Result<Credentials>::Ok(c);
  return Result<Credentials>::Err(Status::Err(
      have && !error.empty() ? error : "NoCredentialProviders: the supervisor published no credentials in time"));
}

void SlotCredentialsProvider::cancel() {
  // Only the flag: a late stop (a signal after the supervisor unmapped the slots) must not touch
  // the slot. A waiting retrieve() looks at the flag at least every kCancelCheck.
  cancelled_.store(true, std::memory_order_release);
}

void SlotCredentialsProvider::stale(const Credentials& c) {
  Credentials cur;
  std::string error;
  uint64_t gen = 0;
  // the set in the slot is the one the service rejected: no worker signs with it again, and the
  // next retrieve() waits for its replacement (the SDK expires its cache before the retry)
  if (read_credential_slot(slot_, &cur, &error, &gen) && error.empty() && cur.access_key_id == c.access_key_id &&
      cur.session_token == c.session_token && cur.expires_unix_ns == c.expires_unix_ns)
    reject_credentials(slot_, gen);
}

}  // namespace ksa
