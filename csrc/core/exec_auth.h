// client-go credential plugins ("exec" users in a kubeconfig).
//
// The reference builds its Kubernetes client with clientcmd.BuildConfigFromFlags on
// KUBE_CONFIG_PATH (/root/reference/scale/scale.go:32-38, client-go v0.19.4 per go.mod:17).
// client-go's REST transport runs a kubeconfig user's `exec` plugin (for example
// `aws eks get-token` or `aws-iam-authenticator token` on EKS) and uses the ExecCredential it
// prints: a bearer token and/or a client certificate, cached until `expirationTimestamp` and
// re-fetched when the apiserver answers 401 to the cached token. This is that authenticator,
// rebuilt on posix_spawn so the worker threads never call back into Python for a token.
#pragma once

#include <atomic>
#include <cstdint>
#include <condition_variable>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "clock.h"
#include "kube.h"
#include "status.h"

namespace ksa {

struct ExecConfig {
  std::string command;  // PATH lookup unless it contains '/'
  std::vector<std::string> args;
  std::vector<std::pair<std::string, std::string>> env;  // appended to (and overriding) the process env
  std::string api_version;  // client.authentication.k8s.io/v1alpha1 or /v1beta1
  std::string install_hint;
  Nanos timeout = 0;  // 0 = wait forever (client-go); the CLI passes --api-timeout
};

struct ExecCredential {
  std::string token;
  std::string cert_pem, key_pem;
  bool has_expiry = false;
  int64_t expiry_unix_ns = 0;
};

// Validates the apiVersion (client-go: `exec plugin: invalid apiVersion "<v>"`).
Status validate_exec_config(const ExecConfig& cfg);

// Runs the plugin once and parses its ExecCredential. `response_code` != 0 is passed to
// v1alpha1 plugins in KUBERNETES_EXEC_INFO (spec.response.code), as client-go does on 401.
// `abort` (optional): set by another thread, the plugin is killed and the run ends with
// "request canceled" (checked every 20 ms).
Result<ExecCredential> run_exec_plugin(const ExecConfig& cfg, int response_code = 0,
                                       const std::atomic<bool>* abort = nullptr);

class ExecTokenProvider final : public TokenProvider {
 public:
  ExecTokenProvider(ExecConfig cfg, std::shared_ptr<Clock> clock);
  // Cached token, or a fresh run when there is none, it expired, or a 401 invalidated it.
  // Callers that arrive during a run wait for it and share its outcome, its error included, so
  // a hanging or failing plugin costs the queues of a process one run, not one each.
  Result<std::string> token() override;
  void invalidate(const std::string& used) override;
  // Kills the run in flight, if any (a stopping client): it and its waiters end with
  // "request canceled"; the cached credential, if any, stays.
  void cancel() override;
  // The whole current credential (client certificate included), refreshed like token().
  Result<ExecCredential> credential();
  uint64_t runs() const;

 private:
  Result<ExecCredential> current();

  ExecConfig cfg_;
  std::shared_ptr<Clock> clock_;
  mutable std::mutex mu_;
  std::condition_variable ran_;  // a run finished (finished_ moved on)
  bool have_ = false;
  int pending_code_ = 0;  // 401 seen on the cached token
  ExecCredential cached_;
  bool running_ = false;
  std::atomic<bool> abort_{false};  // cancel() of the run in flight
  uint64_t finished_ = 0;
  Result<ExecCredential> last_;  // the outcome of the last run
  uint64_t runs_ = 0;
};

}  // namespace ksa
