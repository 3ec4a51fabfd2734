#include "mem_fakes.h"

#include <algorithm>

namespace ksa {

// ---------------------------------------------------------------------------------------
// MockSqsApi / TraceSqsApi

MockSqsApi::MockSqsApi(AttrMap initial) : attrs_(std::move(initial)) {}

Result<AttrMap> MockSqsApi::get_queue_attributes(const std::string&,
                                                 const std::vector<std::string>&) {
  std::lock_guard<std::mutex> lk(mu_);
  calls_++;
  if (clock_) clock_->advance(latency_);
  if (fail_n_ > 0) {
    fail_n_--;
    return Result<AttrMap>::Err(Status::Err(fail_msg_));
  }
  return Result<AttrMap>::Ok(attrs_);
}

void MockSqsApi::set_attributes(AttrMap attrs) {
  std::lock_guard<std::mutex> lk(mu_);
  attrs_ = std::move(attrs);
}

void MockSqsApi::set_latency(std::shared_ptr<VirtualClock> clock, Nanos per_call) {
  std::lock_guard<std::mutex> lk(mu_);
  clock_ = std::move(clock);
  latency_ = per_call;
}

void MockSqsApi::fail_next(int n, std::string message) {
  std::lock_guard<std::mutex> lk(mu_);
  fail_n_ = n;
  fail_msg_ = std::move(message);
}

uint64_t MockSqsApi::calls() const {
  std::lock_guard<std::mutex> lk(mu_);
  return calls_;
}

TraceSqsApi::TraceSqsApi(std::shared_ptr<Clock> clock,
                         std::vector<std::pair<Nanos, AttrMap>> segments, Nanos per_call_latency)
    : clock_(std::move(clock)), segments_(std::move(segments)), latency_(per_call_latency) {
  std::stable_sort(segments_.begin(), segments_.end(),
                   [](const auto& a, const auto& b) { return a.first < b.first; });
}

Result<AttrMap> TraceSqsApi::get_queue_attributes(const std::string&,
                                                  const std::vector<std::string>&) {
  // Sampled at call start, then the call "takes" latency_.
  Nanos t = clock_->now();
  AttrMap cur;
  for (auto& seg : segments_) {
    if (seg.first <= t) cur = seg.second;
    else break;
  }
  if (latency_ > 0) clock_->sleep(latency_, nullptr);
  return Result<AttrMap>::Ok(std::move(cur));
}

// ---------------------------------------------------------------------------------------
// FakeDeployments

FakeDeployments::FakeDeployments(std::string namespace_) : ns_(std::move(namespace_)) {}

void FakeDeployments::add(const std::string& name, int32_t replicas) {
  std::lock_guard<std::mutex> lk(mu_);
  Obj o;
  o.replicas = replicas;
  o.rv = ++rv_counter_;
  objs_[name] = o;
}

void FakeDeployments::add_without_replicas(const std::string& name) {
  std::lock_guard<std::mutex> lk(mu_);
  Obj o;
  o.has_replicas = false;
  o.rv = ++rv_counter_;
  objs_[name] = o;
}

Result<ScaleObject> FakeDeployments::get_locked(const std::string& name) {
  gets_++;
  if (fail_get_ > 0) {
    fail_get_--;
    return Result<ScaleObject>::Err(Status::Err(fail_get_msg_, 500));
  }
  auto it = objs_.find(name);
  if (it == objs_.end())
    return Result<ScaleObject>::Err(Status::Err("deployments.apps \"" + name + "\" not found", 404));
  ScaleObject o;
  o.has_replicas = it->second.has_replicas;
  o.replicas = it->second.replicas;
  o.resource_version = std::to_string(it->second.rv);
  if (conflict_ > 0) {
    conflict_--;
    it->second.rv = ++rv_counter_;  // a concurrent writer (e.g. the deployment controller)
  }
  return Result<ScaleObject>::Ok(o);
}

Result<ScaleObject> FakeDeployments::get(const std::string& name) {
  std::lock_guard<std::mutex> lk(mu_);
  if (clock_) clock_->advance(latency_);
  return get_locked(name);
}

void FakeDeployments::enable_pipelining(bool on) {
  std::lock_guard<std::mutex> lk(mu_);
  pipelining_ = on;
}

bool FakeDeployments::begin_get(const std::string& name, bool) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!pipelining_ || pending_) return false;
  pending_result_ = get_locked(name);  // the server reads the object when the request arrives
  pending_done_at_ = clock_ ? clock_->now() + latency_ : 0;
  pending_ = true;
  return true;
}

Result<ScaleObject> FakeDeployments::finish_get() {
  std::lock_guard<std::mutex> lk(mu_);
  if (!pending_) return Result<ScaleObject>::Err(Status::Err("no pipelined GET in flight"));
  pending_ = false;
  if (clock_ && clock_->now() < pending_done_at_) clock_->advance(pending_done_at_ - clock_->now());
  return pending_result_;
}

Status FakeDeployments::update(const std::string& name, const ScaleObject& fetched,
                               int32_t replicas) {
  std::lock_guard<std::mutex> lk(mu_);
  updates_++;
  if (clock_) clock_->advance(latency_);
  if (fail_update_ > 0) {
    fail_update_--;
    return Status::Err(fail_update_msg_, 500);
  }
  auto it = objs_.find(name);
  if (it == objs_.end()) return Status::Err("deployments.apps \"" + name + "\" not found", 404);
  if (!fetched.resource_version.empty() && fetched.resource_version != std::to_string(it->second.rv))
    return Status::Err("Operation cannot be fulfilled on deployments.apps \"" + name +
                           "\": the object has been modified; please apply your changes to the "
                           "latest version and try again",
                       409);
  it->second.has_replicas = true;
  it->second.replicas = replicas;
  it->second.rv = ++rv_counter_;
  return Status::OK();
}

int32_t FakeDeployments::replicas(const std::string& name) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = objs_.find(name);
  return it == objs_.end() ? -1 : it->second.replicas;
}

void FakeDeployments::set_replicas(const std::string& name, int32_t r) {
  std::lock_guard<std::mutex> lk(mu_);
  auto& o = objs_[name];
  o.has_replicas = true;
  o.replicas = r;
  o.rv = ++rv_counter_;
}

void FakeDeployments::set_latency(std::shared_ptr<VirtualClock> clock, Nanos per_call) {
  std::lock_guard<std::mutex> lk(mu_);
  clock_ = std::move(clock);
  latency_ = per_call;
}

void FakeDeployments::fail_next_get(int n, std::string message) {
  std::lock_guard<std::mutex> lk(mu_);
  fail_get_ = n;
  fail_get_msg_ = std::move(message);
}

void FakeDeployments::fail_next_update(int n, std::string message) {
  std::lock_guard<std::mutex> lk(mu_);
  fail_update_ = n;
  fail_update_msg_ = std::move(message);
}

void FakeDeployments::conflict_next(int n) {
  std::lock_guard<std::mutex> lk(mu_);
  conflict_ = n;
}

uint64_t FakeDeployments::gets() const {
  std::lock_guard<std::mutex> lk(mu_);
  return gets_;
}

uint64_t FakeDeployments::updates() const {
  std::lock_guard<std::mutex> lk(mu_);
  return updates_;
}

}  // namespace ksa
