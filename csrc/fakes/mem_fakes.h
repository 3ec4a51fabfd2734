// In-process fakes of the two API seams the control loop talks through (SqsApi, DeploymentApi):
// the reference's MockSQS (/root/reference/sqs/sqs_test.go:27-59, main_test.go:273-304) and
// client-go's fake clientset (/root/reference/scale/scale_test.go:85-115). Tests and the
// decision-parity harness only: linked into _ksa_fakes, never into _ksa_native.
#pragma once

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../core/clock.h"
#include "../core/kube.h"
#include "../core/sqs.h"

namespace ksa {

// In-memory fake, the MockSQS of /root/reference/sqs/sqs_test.go:27-59: returns the stored
// attribute map; set_attributes() is the SetQueueAttributes test hook. Optionally advances
// a VirtualClock per call (API latency model) and injects failures.
class MockSqsApi final : public SqsApi {
 public:
  explicit MockSqsApi(AttrMap initial = {});
  Result<AttrMap> get_queue_attributes(const std::string& queue_url,
                                       const std::vector<std::string>& names) override;
  void set_attributes(AttrMap attrs);
  void set_latency(std::shared_ptr<VirtualClock> clock, Nanos per_call);
  // The next `n` calls fail with `message`.
  void fail_next(int n, std::string message);
  uint64_t calls() const;

 private:
  mutable std::mutex mu_;
  AttrMap attrs_;
  std::shared_ptr<VirtualClock> clock_;
  Nanos latency_ = 0;
  int fail_n_ = 0;
  std::string fail_msg_;
  uint64_t calls_ = 0;
};

// Time-driven fake: the attribute map is a piecewise-constant function of the clock
// (segments sorted by start time). The decision-parity harness drives the reference's
// synthetic traces through this.
class TraceSqsApi final : public SqsApi {
 public:
  TraceSqsApi(std::shared_ptr<Clock> clock, std::vector<std::pair<Nanos, AttrMap>> segments,
              Nanos per_call_latency);
  Result<AttrMap> get_queue_attributes(const std::string& queue_url,
                                       const std::vector<std::string>& names) override;

 private:
  std::shared_ptr<Clock> clock_;
  std::vector<std::pair<Nanos, AttrMap>> segments_;
  Nanos latency_;
};

// In-memory object tracker (client-go fake clientset equivalent).
class FakeDeployments final : public DeploymentApi {
 public:
  explicit FakeDeployments(std::string namespace_ = "namespace");
  void add(const std::string& name, int32_t replicas);
  void add_without_replicas(const std::string& name);
  Result<ScaleObject> get(const std::string& name) override;
  Status update(const std::string& name, const ScaleObject& fetched, int32_t replicas) override;
  // Pipelined read in virtual time: the snapshot is taken when the GET starts, and
  // finish_get() only advances a VirtualClock to start + latency (the GET ran concurrently with
  // whatever the caller did in between). Disabled unless enable_pipelining(true).
  bool begin_get(const std::string& name, bool may_dial = true) override;
  Result<ScaleObject> finish_get() override;
  void enable_pipelining(bool on);

  int32_t replicas(const std::string& name) const;  // -1 if absent
  void set_replicas(const std::string& name, int32_t r);  // out-of-band edit (kubectl scale)
  void set_latency(std::shared_ptr<VirtualClock> clock, Nanos per_call);
  void fail_next_get(int n, std::string message);
  void fail_next_update(int n, std::string message);
  // Simulates a concurrent writer: bump resourceVersion right after each of the next n GETs,
  // so the following update conflicts (409).
  void conflict_next(int n);
  uint64_t gets() const;
  uint64_t updates() const;

 private:
  struct Obj {
    bool has_replicas = true;
    int32_t replicas = 0;
    uint64_t rv = 1;
  };
  mutable std::mutex mu_;
  std::string ns_;
  std::map<std::string, Obj> objs_;
  std::shared_ptr<VirtualClock> clock_;
  Nanos latency_ = 0;
  int fail_get_ = 0, fail_update_ = 0, conflict_ = 0;
  std::string fail_get_msg_, fail_update_msg_;
  uint64_t gets_ = 0, updates_ = 0;
  uint64_t rv_counter_ = 1000;
  bool pipelining_ = false;
  bool pending_ = false;
  Nanos pending_done_at_ = 0;
  Result<ScaleObject> pending_result_;
  Result<ScaleObject> get_locked(const std::string& name);
};

}  // namespace ksa
