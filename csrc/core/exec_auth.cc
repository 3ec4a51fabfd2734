#include "exec_auth.h"

#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <map>

#include "goutil.h"
#include "json.h"

extern char** environ;

namespace ksa {

namespace {

constexpr const char* kV1Alpha1 = "client.authentication.k8s.io/v1alpha1";
constexpr const char* kV1Beta1 = "client.authentication.k8s.io/v1beta1";

// KUBERNETES_EXEC_INFO: client-go sends it to v1alpha1 plugins only ("input spec disabled for
// beta due to lack of use"); interactive=false is omitted (omitempty), as is a zero code.
std::string exec_info(const ExecConfig& cfg, int response_code, bool interactive) {
  std::string spec;
  if (response_code) spec += "\"response\":{\"code\":" + std::to_string(response_code) + "}";
  if (interactive) spec += std::string(spec.empty() ? "" : ",") + "\"interactive\":true";
  return "{\"kind\":\"ExecCredential\",\"apiVersion\":" + json_quote(cfg.api_version) + ",\"spec\":{" + spec + "}}";
}

std::vector<std::string> build_env(const ExecConfig& cfg, int response_code, bool interactive) {
  // os.Environ() followed by the kubeconfig entries; Go's exec keeps the LAST value of a
  // duplicated key, so the kubeconfig wins.
  std::map<std::string, size_t> pos;
  std::vector<std::string> out;
  auto put = [&](const std::string& k, const std::string& v) {
    auto it = pos.find(k);
    if (it != pos.end()) {
      out[it->second] = k + "=" + v;
    } else {
      pos[k] = out.size();
      out.push_back(k + "=" + v);
    }
  };
  for (char** e = environ; e && *e; ++e) {
    const char* eq = std::strchr(*e, '=');
    if (!eq) continue;
    put(std::string(*e, static_cast<size_t>(eq - *e)), std::string(eq + 1));
  }
  for (const auto& kv : cfg.env) put(kv.first, kv.second);
  if (cfg.api_version == kV1Alpha1) put("KUBERNETES_EXEC_INFO", exec_info(cfg, response_code, interactive));
  return out;
}

Status not_found(const ExecConfig& cfg) {
  std::string m = "exec: executable " + cfg.command + " not found";
  m += "\n\nIt looks like you are trying to use a client-go credential plugin that is not installed.";
  if (!cfg.install_hint.empty()) m += "\n\n" + cfg.install_hint;
  return Status::Err(m);
}

Result<ExecCredential> parse_exec_credential(const ExecConfig& cfg, const std::string& out) {
  auto j = json_parse(out);
  if (!j.ok() || !j.value.is_object()) {
    return Result<ExecCredential>::Err(
        Status::Err("decoding stdout: " + (j.ok() ? std::string("not a JSON object") : j.status.message())));
  }
  const JsonValue* kind = j.value.get("kind");
  const JsonValue* apiv = j.value.get("apiVersion");
  if (!kind || !kind->is_string() || kind->str.empty())
    return Result<ExecCredential>::Err(Status::Err("decoding stdout: Object 'Kind' is missing in '" + out + "'"));
  const std::string got = apiv && apiv->is_string() ? apiv->str : "";
  if (got != cfg.api_version) {
    return Result<ExecCredential>::Err(Status::Err("exec plugin is configured to use API version " + cfg.api_version +
                                                   ", plugin returned version " + got));
  }
  const JsonValue* st = j.value.get("status");
  if (!st || st->type == JsonValue::Type::Null)
    return Result<ExecCredential>::Err(Status::Err("exec plugin didn't return a status field"));
  ExecCredential c;
  auto str = [&](const char* k) {
    const JsonValue* v = st->get(k);
    return v && v->is_string() ? v->str : std::string();
  };
  c.token = str("token");
  c.cert_pem = str("clientCertificateData");
  c.key_pem = str("clientKeyData");
  if (c.token.empty() && c.cert_pem.empty() && c.key_pem.empty())
    return Result<ExecCredential>::Err(Status::Err("exec plugin didn't return a token or cert/key pair"));
  if (c.cert_pem.empty() != c.key_pem.empty())
    return Result<ExecCredential>::Err(Status::Err("exec plugin returned only certificate or key, not both"));
  const std::string exp = str("expirationTimestamp");
  if (!exp.empty()) {
    if (!parse_rfc3339(exp, &c.expiry_unix_ns))
      return Result<ExecCredential>::Err(Status::Err("decoding stdout: bad expirationTimestamp \"" + exp + "\""));
    c.has_expiry = true;
  }
  return Result<ExecCredential>::Ok(std::move(c));
}

}  // namespace

Status validate_exec_config(const ExecConfig& cfg) {
  if (cfg.api_version != kV1Alpha1 && cfg.api_version != kV1Beta1)
    return Status::Err("exec plugin: invalid apiVersion \"" + cfg.api_version + "\"");
  if (cfg.command.empty()) return Status::Err("exec plugin: command must be specified");
  return Status::OK();
}

Result<ExecCredential> run_exec_plugin(const ExecConfig& cfg, int response_code, const std::atomic<bool>* abort) {
  Status v = validate_exec_config(cfg);
  if (!v.ok()) return Result<ExecCredential>::Err(v);
  const bool interactive = isatty(STDIN_FILENO) == 1;
  std::vector<std::string> env = build_env(cfg, response_code, interactive);
  std::vector<char*> envp;
  for (auto& e : env) envp.push_back(&e[0]);
  envp.push_back(nullptr);
  std::vector<std::string> argv_s;
  argv_s.push_back(cfg.command);
  for (const auto& a : cfg.args) argv_s.push_back(a);
  std::vector<char*> argv;
  for (auto& a : argv_s) argv.push_back(&a[0]);
  argv.push_back(nullptr);

  int fds[2];
  if (pipe2(fds, O_CLOEXEC) != 0) return Result<ExecCredential>::Err(Status::Err(std::string("exec: pipe: ") + std::strerror(errno)));
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_adddup2(&fa, fds[1], STDOUT_FILENO);  // stderr stays the process's
  if (!interactive) posix_spawn_file_actions_addopen(&fa, STDIN_FILENO, "/dev/null", O_RDONLY, 0);
  pid_t pid = -1;
  int rc = posix_spawnp(&pid, cfg.command.c_str(), &fa, nullptr, argv.data(), envp.data());
  posix_spawn_file_actions_destroy(&fa);
  close(fds[1]);
  if (rc != 0) {
    close(fds[0]);
    if (rc == ENOENT || rc == EACCES) return Result<ExecCredential>::Err(not_found(cfg));
    return Result<ExecCredential>::Err(Status::Err("exec: " + cfg.command + ": " + std::strerror(rc)));
  }

  std::string out;
  char buf[4096];
  const int64_t deadline_ms = cfg.timeout > 0 ? cfg.timeout / kMillisecond : -1;
  RealClock rc_clock;
  const Nanos start = rc_clock.now();
  bool timed_out = false, aborted = false;
  for (;;) {
    if (abort && abort->load(std::memory_order_acquire)) {
      aborted = true;
      break;
    }
    int wait_ms = abort ? 20 : -1;
    if (deadline_ms >= 0) {
      const int64_t left = deadline_ms - (rc_clock.now() - start) / kMillisecond;
      if (left <= 0) {
        timed_out = true;
        break;
      }
      wait_ms = wait_ms < 0 ? static_cast<int>(left) : static_cast<int>(std::min<int64_t>(left, wait_ms));
    }
    struct pollfd p = {fds[0], POLLIN, 0};
    int pr = poll(&p, 1, wait_ms);
    if (pr < 0) {
      if (errno == EINTR) continue;
      break;
    }
    if (pr == 0) continue;  // re-check the deadline
    ssize_t n = read(fds[0], buf, sizeof buf);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) break;
    out.append(buf, static_cast<size_t>(n));
  }
  close(fds[0]);
  if (timed_out || aborted) kill(pid, SIGKILL);
  int status = 0;
  while (waitpid(pid, &status, 0) < 0 && errno == EINTR) {
  }
  if (aborted) return Result<ExecCredential>::Err(Status::Err("request canceled"));
  if (timed_out) {
    return Result<ExecCredential>::Err(Status::Err("exec: executable " + cfg.command + " timed out after " +
                                                   std::to_string(cfg.timeout / kMillisecond) + "ms"));
  }
  if (WIFEXITED(status) && WEXITSTATUS(status) == 127 && out.empty()) return Result<ExecCredential>::Err(not_found(cfg));
  if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) {
    const int code = WIFEXITED(status) ? WEXITSTATUS(status) : -1;
    return Result<ExecCredential>::Err(
        Status::Err("exec: executable " + cfg.command + " failed with exit code " + std::to_string(code)));
  }
  return parse_exec_credential(cfg, out);
}

ExecTokenProvider::ExecTokenProvider(ExecConfig cfg, std::shared_ptr<Clock> clock)
    : cfg_(std::move(cfg)), clock_(std::move(clock)) {}

Result<ExecCredential> ExecTokenProvider::current() {
  std::unique_lock<std::mutex> lk(mu_);
  // client-go: reuse the cached credential unless it expired (strict After, a zero expiry
  // never expires) or a 401 on it asked for a refresh.
  if (have_ && pending_code_ == 0 && (!cached_.has_expiry || clock_->unix_nanos() <= cached_.expiry_unix_ns))
    return Result<ExecCredential>::Ok(cached_);
  if (running_) {  // another queue runs the plugin: its outcome is this caller's too
    const uint64_t ticket = finished_;
    ran_.wait(lk, [&] { return finished_ != ticket; });
    return last_;
  }
  running_ = true;
  abort_.store(false, std::memory_order_relaxed);
  const int code = pending_code_;
  ++runs_;
  lk.unlock();
  Result<ExecCredential> r;
  try {
    r = run_exec_plugin(cfg_, code, &abort_);
  } catch (const std::exception& e) {  // the waiters must be released whatever happens
    r = Result<ExecCredential>::Err(Status::Err(e.what()));
  }
  lk.lock();
  running_ = false;
  if (!r.ok()) {
    if (r.status.message() != "request canceled") r = Result<ExecCredential>::Err(r.status.wrap("getting credentials"));
  } else {
    cached_ = r.value;
    have_ = true;
    pending_code_ = 0;  // a 401 reported during the run was about the token this one replaces
  }
  last_ = r;
  ++finished_;
  ran_.notify_all();
  return r;
}

Result<ExecCredential> ExecTokenProvider::credential() { return current(); }

Result<std::string> ExecTokenProvider::token() {
  auto c = current();
  if (!c.ok()) return Result<std::string>::Err(c.status);
  return Result<std::string>::Ok(c.value.token);
}

void ExecTokenProvider::cancel() {
  std::lock_guard<std::mutex> lk(mu_);
  if (running_) abort_.store(true, std::memory_order_release);
}

void ExecTokenProvider::invalidate(const std::string& used) {
  std::lock_guard<std::mutex> lk(mu_);
  if (have_ && cached_.token == used) pending_code_ = 401;
}

uint64_t ExecTokenProvider::runs() const {
  std::lock_guard<std::mutex> lk(mu_);
  return runs_;
}

}  // namespace ksa
