// Python bindings for the native autoscaler runtime (`kube_sqs_autoscaler_amd.ops._ksa_native`).
//
// Python owns configuration and bootstrap (Go-compatible flag parsing, the AWS credential
// chain, kubeconfig / in-cluster discovery); everything on the poll -> patch path runs here in
// C++ with the GIL released. The injectable seams of the reference -- the `SQS` interface
// (/root/reference/sqs/sqs.go:14-18) and typedappv1.DeploymentInterface
// (/root/reference/scale/scale.go:22) -- are exposed as subclassable base classes
// (SqsApi, DeploymentApi), so Python fakes plug into the native loop exactly like the
// reference's Go mocks plug into Run(). The native fakes (localhost endpoints, in-memory
// MockSqsApi / FakeDeployments) are a separate module, _ksa_fakes (fakes_module.cc), that tests,
// benchmarks and the parity harness load; this one is what the image ships.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <unistd.h>

#include "../core/clock.h"
#include "../core/cred_slot.h"
#include "../core/exec_auth.h"
#include "../core/goutil.h"
#include "../core/http.h"
#include "../core/json.h"
#include "../core/kube.h"
#include "../core/log.h"
#include "../core/runner.h"
#include "../core/sigv4.h"
#include "../core/sqs.h"
#include "../core/sweep.h"
#include "../core/xml.h"

namespace py = pybind11;
using namespace ksa;

namespace {

py::object g_native_error;  // kube_sqs_autoscaler_amd.ops._ksa_native.NativeError

[[noreturn]] void raise_status(const Status& s) {
  PyErr_SetString(g_native_error.ptr(), s.message().c_str());
  throw py::error_already_set();
}

template <class T>
T unwrap(Result<T> r) {
  if (!r.ok()) raise_status(r.status);
  return std::move(r.value);
}

std::string py_error_text(py::error_already_set& e) {
  py::gil_scoped_acquire g;
  std::string msg = py::str(e.value());
  return msg;
}

// ---- trampolines ------------------------------------------------------------------------

class PySqsApi : public SqsApi, public py::trampoline_self_life_support {
 public:
  Result<AttrMap> get_queue_attributes(const std::string& queue_url,
                                       const std::vector<std::string>& names) override {
    py::gil_scoped_acquire g;
    py::function f = py::get_override(static_cast<const SqsApi*>(this), "get_queue_attributes");
    if (!f) return Result<AttrMap>::Err(Status::Err("SqsApi.get_queue_attributes not implemented"));
    try {
      py::object r = f(queue_url, names);
      AttrMap out;
      for (auto item : r.cast<py::dict>())
        out[py::str(item.first)] = py::str(item.second);
      return Result<AttrMap>::Ok(std::move(out));
    } catch (py::error_already_set& e) {
      return Result<AttrMap>::Err(Status::Err(py_error_text(e)));
    }
  }
};

class PyDeploymentApi : public DeploymentApi, public py::trampoline_self_life_support {
 public:
  Result<ScaleObject> get(const std::string& name) override {
    py::gil_scoped_acquire g;
    py::function f = py::get_override(static_cast<const DeploymentApi*>(this), "get");
    if (!f) return Result<ScaleObject>::Err(Status::Err("DeploymentApi.get not implemented"));
    try {
      return Result<ScaleObject>::Ok(f(name).cast<ScaleObject>());
    } catch (py::error_already_set& e) {
      return Result<ScaleObject>::Err(Status::Err(py_error_text(e)));
    }
  }
  Status update(const std::string& name, const ScaleObject& fetched, int32_t replicas) override {
    py::gil_scoped_acquire g;
    py::function f = py::get_override(static_cast<const DeploymentApi*>(this), "update");
    if (!f) return Status::Err("DeploymentApi.update not implemented");
    try {
      f(name, fetched, replicas);
      return Status::OK();
    } catch (py::error_already_set& e) {
      return Status::Err(py_error_text(e));
    }
  }
};

class PyCredentialsProvider : public CredentialsProvider, public py::trampoline_self_life_support {
 public:
  Result<Credentials> retrieve() override {
    py::gil_scoped_acquire g;
    py::function f = py::get_override(static_cast<const CredentialsProvider*>(this), "retrieve");
    if (!f) return Result<Credentials>::Err(Status::Err("CredentialsProvider.retrieve not implemented"));
    try {
      return Result<Credentials>::Ok(f().cast<Credentials>());
    } catch (py::error_already_set& e) {
      return Result<Credentials>::Err(Status::Err(py_error_text(e)));
    }
  }
};

class PyTokenProvider : public TokenProvider, public py::trampoline_self_life_support {
 public:
  Result<std::string> token() override {
    py::gil_scoped_acquire g;
    py::function f = py::get_override(static_cast<const TokenProvider*>(this), "token");
    if (!f) return Result<std::string>::Err(Status::Err("TokenProvider.token not implemented"));
    try {
      return Result<std::string>::Ok(f().cast<std::string>());
    } catch (py::error_already_set& e) {
      return Result<std::string>::Err(Status::Err(py_error_text(e)));
    }
  }
};

Level level_from(const std::string& s) {
  Level l;
  if (!parse_level(s, &l)) throw py::value_error("not a valid logrus Level: " + s);
  return l;
}

py::dict record_dict(const IterationRecord& r) {
  py::dict d;
  d["index"] = r.index;
  d["stopped"] = r.stopped;
  d["t_poll"] = r.t_poll;
  d["depth_ok"] = r.depth_ok;
  d["depth"] = r.depth;
  d["up"] = action_name(r.up);
  d["down"] = action_name(r.down);
  d["replicas_before"] = r.replicas_before;
  d["replicas_after"] = r.replicas_after;
  d["prefetched"] = r.prefetched;
  d["prefetch_used"] = r.prefetch_used;
  d["prefetch_gated"] = r.prefetch_gated;
  d["gets"] = r.gets;
  d["depth_ns"] = r.depth_ns;
  d["get_ns"] = r.get_ns;
  d["update_ns"] = r.update_ns;
  d["total_ns"] = r.total_ns;
  d["patch_latency_ns"] = r.patch_latency_ns;
  d["cpu_ns"] = r.cpu_ns;
  d["error"] = r.error;
  return d;
}

py::dict http_stats_dict(const HttpClientStats& s) {
  py::dict d;
  d["requests"] = s.requests;
  d["connects"] = s.connects;
  d["tls_resumptions"] = s.tls_resumptions;
  d["reconnect_retries"] = s.reconnect_retries;
  d["idle_closed"] = s.idle_closed;
  d["presends"] = s.presends;
  d["presend_discards"] = s.presend_discards;
  d["bytes_out"] = s.bytes_out;
  d["bytes_in"] = s.bytes_in;
  d["tls_version"] = s.tls_version;
  d["tls_cipher"] = s.tls_cipher;
  return d;
}

Headers headers_from(const py::object& o) {
  Headers h;
  if (o.is_none()) return h;
  if (py::isinstance<py::dict>(o)) {
    for (auto item : o.cast<py::dict>()) h.emplace_back(py::str(item.first), py::str(item.second));
    return h;
  }
  for (auto item : o) {
    auto t = item.cast<py::tuple>();
    h.emplace_back(t[0].cast<std::string>(), t[1].cast<std::string>());
  }
  return h;
}

}  // namespace

PYBIND11_MODULE(_ksa_native, m) {
  m.doc() = "Native runtime of the MI355X SQS autoscaler (control loop, SigV4, HTTP/TLS, SQS + kube clients).";
  g_native_error = py::reinterpret_borrow<py::object>(
      PyErr_NewException("kube_sqs_autoscaler_amd.ops._ksa_native.NativeError", PyExc_RuntimeError, nullptr));
  m.attr("NativeError") = g_native_error;

  // ---- Go stdlib helpers ----
  m.def("go_atoi", [](const std::string& s) { return unwrap(go_atoi(s)); });
  m.def("go_quote", &go_quote);
  m.def("rfc3339_utc", &rfc3339_utc);
  m.def("amz_date", &amz_date);
  m.def("go_int32", &go_int32);

  // ---- JSON / XML ----
  m.def("set_spec_replicas", [](const std::string& raw, int32_t r) { return unwrap(set_spec_replicas(raw, r)); });
  m.def("json_roundtrip", [](const std::string& t) { return json_serialize(unwrap(json_parse(t))); });
  m.def("xml_sqs_attributes", &xml_sqs_attributes);
  m.def("xml_first_text", [](const std::string& doc, const std::string& tag) {
    bool found = false;
    std::string v = xml_first_text(doc, tag, &found);
    return found ? py::object(py::str(v)) : py::object(py::none());
  });

  // ---- crypto / SigV4 ----
  m.def("sha256_hex", [](py::bytes b) { return sha256_hex(std::string(b)); });
  m.def("hmac_sha256_hex", [](py::bytes k, py::bytes d) { return hex_encode(hmac_sha256(std::string(k), std::string(d))); });
  m.def("aws_uri_encode", &aws_uri_encode, py::arg("s"), py::arg("keep_slash") = false);

  py::class_<Credentials>(m, "Credentials")
      .def(py::init([](std::string akid, std::string secret, std::string token, int64_t exp, std::string name) {
             Credentials c;
             c.access_key_id = std::move(akid);
             c.secret_access_key = std::move(secret);
             c.session_token = std::move(token);
             c.expires_unix_ns = exp;
             c.provider_name = std::move(name);
             return c;
           }),
           py::arg("access_key_id"), py::arg("secret_access_key"), py::arg("session_token") = "",
           py::arg("expires_unix_ns") = 0, py::arg("provider_name") = "")
      .def_readwrite("access_key_id", &Credentials::access_key_id)
      .def_readwrite("secret_access_key", &Credentials::secret_access_key)
      .def_readwrite("session_token", &Credentials::session_token)
      .def_readwrite("expires_unix_ns", &Credentials::expires_unix_ns)
      .def_readwrite("provider_name", &Credentials::provider_name)
      .def_readonly("kept_after_failed_refresh", &Credentials::kept_after_failed_refresh)
      .def("valid", &Credentials::valid)
      .def("__repr__", [](const Credentials& c) {
        return "Credentials(access_key_id=" + c.access_key_id + ", provider=" + c.provider_name + ")";
      });

  py::class_<CredentialsProvider, PyCredentialsProvider, py::smart_holder>(m, "CredentialsProvider")
      .def(py::init<>())
      .def("retrieve", [](CredentialsProvider& p) {
        Result<Credentials> r;
        {
          py::gil_scoped_release rel;
          r = p.retrieve();
        }
        return unwrap(r);
      });
  py::class_<StaticCredentialsProvider, CredentialsProvider, py::smart_holder>(m, "StaticCredentialsProvider")
      .def(py::init<Credentials>());
  // ---- the process fleet's shared credential slot (cred_slot.h) ----
  auto cs = [](uintptr_t addr) { return reinterpret_cast<SharedCredentialSlot*>(addr); };
  m.def("credential_slot_size", [] { return sizeof(SharedCredentialSlot); });
  m.def("init_credential_slot", [](uintptr_t addr) { init_credential_slot(reinterpret_cast<void*>(addr)); });
  m.def("publish_credentials", [cs](uintptr_t addr, const Credentials& c, const std::string& refresh_error) {
    publish_credentials(cs(addr), c, refresh_error);
  }, py::arg("addr"), py::arg("creds"), py::arg("refresh_error") = "");
  m.def("publish_credential_error", [cs](uintptr_t addr, const std::string& e) { publish_credential_error(cs(addr), e); });
  m.def("read_credential_slot", [cs](uintptr_t addr) -> py::tuple {
    Credentials c;
    std::string error;
    uint64_t gen = 0;
    if (!read_credential_slot(cs(addr), &c, &error, &gen)) return py::make_tuple(py::none(), std::string(), 0);
    return py::make_tuple(py::cast(c), error, gen);
  });
  m.def("request_credentials", [cs](uintptr_t addr, uint64_t gen) { request_credentials(cs(addr), gen); });
  m.def("reject_credentials", [cs](uintptr_t addr, uint64_t gen) { reject_credentials(cs(addr), gen); });
  m.def("credential_slot_still_signs", [cs](uintptr_t addr, int64_t unix_now, int64_t skew) {
    return credential_slot_still_signs(cs(addr), unix_now, skew);
  });
  // the slot's counters and the refresh error of a set kept after a failed refresh
  m.def("credential_slot_info", [cs](uintptr_t addr) {
    auto* s = cs(addr);
    Credentials c;
    std::string error, refresh_error;
    uint64_t gen = 0;
    read_credential_slot(s, &c, &error, &gen, &refresh_error);
    py::dict d;
    d["generation"] = gen;
    d["wanted"] = s->wanted.load();
    d["rejected"] = s->rejected.load();
    d["stale_signs"] = s->stale_signs.load();
    d["error"] = error;
    d["refresh_error"] = refresh_error;
    return d;
  });
  m.attr("CREDENTIAL_STALE_SKEW_NS") = kStaleSkew;
  m.def("credential_slot_asks", [cs](uintptr_t addr) { return credential_slot_asks(cs(addr)); });
  // the broker's serving thread sleeps here between looks (GIL released): a worker's ask wakes it
  m.def("credential_slot_wait_ask", [cs](uintptr_t addr, uint32_t seen, int64_t timeout_ns) {
    return credential_slot_wait_ask(cs(addr), seen, timeout_ns);
  }, py::call_guard<py::gil_scoped_release>());
  m.def("credential_slot_poke", [cs](uintptr_t addr) { credential_slot_poke(cs(addr)); });
  m.def("credential_slot_needs_fetch", [cs](uintptr_t addr, int64_t unix_now, int64_t window) {
    return credential_slot_needs_fetch(cs(addr), unix_now, window);
  });
  py::class_<SlotCredentialsProvider, CredentialsProvider, py::smart_holder>(m, "SlotCredentialsProvider")
      .def(py::init([cs](uintptr_t addr, std::shared_ptr<Clock> clock, int64_t window_ns, int64_t wait_limit_ns,
                         int64_t skew_ns) {
             return std::make_shared<SlotCredentialsProvider>(cs(addr), [clock] { return clock->unix_nanos(); },
                                                              window_ns, wait_limit_ns, skew_ns);
           }),
           py::arg("addr"), py::arg("clock"), py::arg("expiry_window_ns") = 5LL * 60 * kSecond,
           py::arg("wait_limit_ns") = 15 * kSecond, py::arg("skew_ns") = kStaleSkew)
      .def("stale", &SlotCredentialsProvider::stale, py::call_guard<py::gil_scoped_release>())
      .def("cancel", &SlotCredentialsProvider::cancel);
  py::class_<SharedCredentialsProvider, CredentialsProvider, py::smart_holder>(m, "SharedCredentialsProvider")
      .def(py::init([](std::shared_ptr<CredentialsProvider> inner, std::shared_ptr<Clock> clock, int64_t window_ns) {
             return std::make_shared<SharedCredentialsProvider>(
                 std::move(inner), [clock] { return clock->unix_nanos(); }, window_ns);
           }),
           py::arg("inner"), py::arg("clock"), py::arg("expiry_window_ns") = 5LL * 60 * kSecond)
      // the lock may be held by a fetch waiting for the GIL (a Python inner provider)
      .def("fetches", &SharedCredentialsProvider::fetches, py::call_guard<py::gil_scoped_release>())
      .def("stale_signs", &SharedCredentialsProvider::stale_signs)
      .def("stale", &SharedCredentialsProvider::stale, py::call_guard<py::gil_scoped_release>())
      .def("cancel", &SharedCredentialsProvider::cancel, py::call_guard<py::gil_scoped_release>());

  py::class_<SigV4Signer, std::shared_ptr<SigV4Signer>>(m, "SigV4Signer")
      .def(py::init<std::string, std::string>(), py::arg("region"), py::arg("service"))
      .def("sign",
           [](SigV4Signer& s, const Credentials& c, int64_t unix_ns, const std::string& method,
              const std::string& path, const std::string& query, py::object headers, py::bytes body) {
             Headers h = headers_from(headers);
             SignDebug dbg;
             s.sign(c, unix_ns, method, path, query, &h, std::string(body), &dbg);
             py::dict d;
             d["canonical_request"] = dbg.canonical_request;
             d["string_to_sign"] = dbg.string_to_sign;
             d["signed_headers"] = dbg.signed_headers;
             d["signature"] = dbg.signature;
             d["scope"] = dbg.scope;
             return py::make_tuple(h, d);
           })
      .def("sign_prepared",
           [](SigV4Signer& s, const Credentials& c, int64_t unix_ns, const std::string& method,
              const std::string& path, const std::string& query, py::object headers, py::bytes body) {
             // prepare() + sign_prepared(): the per-queue fast path HttpSqsApi uses
             SigV4Prepared p = s.prepare(method, path, query, headers_from(headers), std::string(body));
             Headers h;
             SignDebug dbg;
             s.sign_prepared(p, c, unix_ns, &h, &dbg);
             py::dict d;
             d["canonical_request"] = dbg.canonical_request;
             d["string_to_sign"] = dbg.string_to_sign;
             d["signed_headers"] = dbg.signed_headers;
             d["signature"] = dbg.signature;
             return py::make_tuple(h, d);
           })
      .def("sign_prepared_headers",
           [](SigV4Signer& s, const Credentials& c, int64_t unix_ns, const std::string& method,
              const std::string& path, const std::string& query, py::object headers, py::bytes body) {
             // exactly what HttpSqsApi does per poll (no debug capture: the in-place fast path)
             SigV4Prepared p = s.prepare(method, path, query, headers_from(headers), std::string(body));
             Headers h;
             s.sign_prepared(p, c, unix_ns, &h, nullptr);
             return h;
           })
      .def("signing_key_hex", [](SigV4Signer& s, const std::string& secret, const std::string& date) {
        return hex_encode(s.signing_key(secret, date));
      });
  m.def("sigv4_verify",
        [](const std::string& method, const std::string& path, const std::string& query, py::object headers,
           py::bytes body, const std::string& akid, const std::string& secret, const std::string& region,
           const std::string& service) {
          Status s = sigv4_verify(method, path, query, headers_from(headers), std::string(body), akid, secret,
                                  region, service);
          if (!s.ok()) raise_status(s);
        });

  // ---- logging ----
  py::class_<Logger, std::shared_ptr<Logger>>(m, "Logger")
      .def(py::init<>())
      .def_static("default", &Logger::default_logger)
      .def("set_level", [](Logger& l, const std::string& s) { l.set_level(level_from(s)); })
      .def("level", [](Logger& l) { return std::string(level_name(l.level())); })
      .def("set_format", [](Logger& l, const std::string& f) {
        if (f == "text") l.set_format(LogFormat::Text);
        else if (f == "json") l.set_format(LogFormat::Json);
        else if (f == "text-color") l.set_format(LogFormat::TextColor);
        else throw py::value_error("log format must be text or json");
      })
      .def("set_base_time", &Logger::set_base_time, py::arg("unix_ns"))
      .def("set_sink",
           [](Logger& l, py::object cb) {
             if (cb.is_none()) {
               l.set_sink_fd(2);
               return;
             }
             auto holder = std::make_shared<py::object>(cb);
             l.set_sink([holder](const std::string& line) {
               py::gil_scoped_acquire g;
               try {
                 (*holder)(line);
               } catch (py::error_already_set& e) {
                 e.discard_as_unraisable(__func__);
               }
             });
           })
      .def("set_sink_fd",
           [](Logger& l, int fd) {
             // Native fd sink (no GIL): one write(2) per line, like logrus on os.Stderr.
             l.set_sink_fd(fd);
           })
      .def("set_time_source",
           [](Logger& l, std::shared_ptr<Clock> c) {
             l.set_time_source([c] { return c->unix_nanos(); });
           })
      .def("set_base_fields", &Logger::set_base_fields)
      .def("with_fields", &Logger::with_fields)
      .def("log",
           [](Logger& l, const std::string& level, const std::string& msg, const Fields& f) {
             l.log(level_from(level), msg, f);
           },
           py::arg("level"), py::arg("msg"), py::arg("fields") = Fields{},
           py::call_guard<py::gil_scoped_release>())
      .def("format", [](Logger& l, const std::string& level, const std::string& msg, const Fields& f,
                        int64_t ts) { return l.format(level_from(level), msg, f, ts); });
  m.def("logrus_needs_quoting", &logrus_needs_quoting);

  // ---- clocks ----
  py::class_<Clock, std::shared_ptr<Clock>>(m, "Clock")
      .def("now", &Clock::now)
      .def("unix_nanos", &Clock::unix_nanos)
      .def("sleep", [](Clock& c, Nanos d) { return c.sleep(d, nullptr); }, py::call_guard<py::gil_scoped_release>());
  py::class_<RealClock, Clock, std::shared_ptr<RealClock>>(m, "RealClock").def(py::init<>());
  py::class_<VirtualClock, Clock, std::shared_ptr<VirtualClock>>(m, "VirtualClock")
      .def(py::init<Nanos, int64_t>(), py::arg("start") = 0, py::arg("unix_epoch_ns") = 1700000000LL * kSecond)
      .def("advance", &VirtualClock::advance)
      .def("set", &VirtualClock::set);

  // ---- HTTP ----
  py::class_<TlsOptions>(m, "TlsOptions")
      .def(py::init<>())
      .def_readwrite("insecure_skip_verify", &TlsOptions::insecure_skip_verify)
      .def_readwrite("ca_file", &TlsOptions::ca_file)
      .def_readwrite("ca_pem", &TlsOptions::ca_pem)
      .def_readwrite("cert_pem", &TlsOptions::cert_pem)
      .def_readwrite("key_pem", &TlsOptions::key_pem)
      .def_readwrite("server_name", &TlsOptions::server_name);

  py::class_<HttpClient, std::shared_ptr<HttpClient>>(m, "HttpClient")
      .def(py::init([](const std::string& url, const TlsOptions& tls, Nanos timeout) {
             return std::make_shared<HttpClient>(unwrap(parse_url(url)), tls, timeout);
           }),
           py::arg("origin"), py::arg("tls") = TlsOptions(), py::arg("timeout_ns") = 30 * kSecond)
      .def("request",
           [](HttpClient& c, const std::string& method, const std::string& target, py::object headers,
              py::bytes body, Nanos timeout) {
             HttpRequest req;
             req.method = method;
             req.target = target;
             req.headers = headers_from(headers);
             req.body = std::string(body);
             HttpResponse resp;
             Status s;
             {
               py::gil_scoped_release rel;
               s = c.round_trip(req, &resp, timeout);
             }
             if (!s.ok()) raise_status(s);
             return py::make_tuple(resp.status, resp.headers, py::bytes(resp.body));
           },
           py::arg("method"), py::arg("target"), py::arg("headers") = py::none(), py::arg("body") = py::bytes(""),
           py::arg("timeout_ns") = -1)
      .def("set_busy_poll", &HttpClient::set_busy_poll)
      .def("warm", &HttpClient::warm, py::arg("dial_budget_ns") = HttpClient::kWarmDialBudget,
           py::call_guard<py::gil_scoped_release>())
      .def("stage",
           [](HttpClient& c, const std::string& method, const std::string& target, py::object headers,
              py::bytes body) {
             HttpRequest req;
             req.method = method;
             req.target = target;
             req.headers = headers_from(headers);
             req.body = std::string(body);
             return c.stage(req);
           },
           py::arg("method"), py::arg("target"), py::arg("headers") = py::none(), py::arg("body") = py::bytes(""))
      .def("set_proxy",
           [](HttpClient& c, const std::string& url) {
             Status s = c.set_proxy(url);
             if (!s.ok()) raise_status(s);
           })
      .def_property_readonly("proxied", &HttpClient::proxied)
      .def("rtt_ewma", &HttpClient::rtt_ewma)
      .def("close", &HttpClient::close)
      .def("stats", [](HttpClient& c) { return http_stats_dict(c.stats()); });
  auto quota_tuple = [](const CpuQuota& q) { return py::make_tuple(q.quota_ns, q.period_ns); };
  m.def("parse_cpu_max", [quota_tuple](const std::string& t) { return quota_tuple(parse_cpu_max(t)); });
  m.def("parse_cfs_quota", [quota_tuple](const std::string& q, const std::string& p) {
    return quota_tuple(parse_cfs_quota(q, p));
  });
  m.def("read_cpu_quota", [quota_tuple](const std::string& root) { return quota_tuple(read_cpu_quota(root)); },
        py::arg("root") = "/sys/fs/cgroup");
  m.def("runner_spin_budget", [](const LoopConfig& cfg, int64_t quota_ns, int64_t period_ns) {
    CpuQuota q;
    q.quota_ns = quota_ns;
    q.period_ns = period_ns;
    return Runner::spin_budget_for(cfg, q);
  }, py::arg("config"), py::arg("quota_ns") = 0, py::arg("period_ns") = 0);
  m.def("http_spin_window", &HttpClient::spin_window_for, py::arg("busy_poll_ns"), py::arg("ewma_ns"),
        py::arg("budget_ns"));
  m.def("parse_url", [](const std::string& s) {
    Url u = unwrap(parse_url(s));
    return py::make_tuple(u.scheme, u.host, u.port, u.path);
  });
  // ---- SQS ----
  m.def("default_attribute_names", &default_attribute_names);
  py::enum_<SqsProtocol>(m, "SqsProtocol").value("Query", SqsProtocol::Query).value("Json", SqsProtocol::Json);
  py::class_<SqsHttpOptions>(m, "SqsHttpOptions")
      .def(py::init<>())
      .def_readwrite("region", &SqsHttpOptions::region)
      .def_readwrite("endpoint", &SqsHttpOptions::endpoint)
      .def_readwrite("protocol", &SqsHttpOptions::protocol)
      .def_readwrite("timeout_ns", &SqsHttpOptions::timeout)
      .def_readwrite("busy_poll_ns", &SqsHttpOptions::busy_poll)
      .def_readwrite("proxy", &SqsHttpOptions::proxy)
      .def_readwrite("max_retries", &SqsHttpOptions::max_retries)
      .def_readwrite("min_retry_delay_ns", &SqsHttpOptions::min_retry_delay)
      .def_readwrite("min_throttle_delay_ns", &SqsHttpOptions::min_throttle_delay)
      .def_readwrite("max_retry_delay_ns", &SqsHttpOptions::max_retry_delay)
      .def_readwrite("tls", &SqsHttpOptions::tls);

  py::class_<SqsApi, PySqsApi, py::smart_holder>(m, "SqsApi")
      .def(py::init<>())
      .def("get_queue_attributes", [](SqsApi& a, const std::string& url, const std::vector<std::string>& names) {
        Result<AttrMap> r;
        {
          py::gil_scoped_release rel;
          r = a.get_queue_attributes(url, names);
        }
        return unwrap(r);
      });
  py::class_<HttpSqsApi, SqsApi, py::smart_holder>(m, "HttpSqsApi")
      .def(py::init<SqsHttpOptions, std::shared_ptr<CredentialsProvider>, std::shared_ptr<Clock>>(),
           py::arg("options"), py::arg("credentials"), py::arg("clock"))
      .def("set_timing", &HttpSqsApi::set_timing)
      .def_static("endpoint_for_region", &HttpSqsApi::endpoint_for_region)
      .def_static("signing_region", &HttpSqsApi::signing_region)
      .def("endpoint", &HttpSqsApi::endpoint)
      .def("stats", [](HttpSqsApi& a) {
        auto s = a.stats();
        py::dict d;
        d["calls"] = s.calls;
        d["retries"] = s.retries;
        d["throttle_retries"] = s.throttle_retries;
        d["errors"] = s.errors;
        d["http"] = http_stats_dict(s.http);
        return d;
      });
  py::class_<SqsClient, std::shared_ptr<SqsClient>>(m, "SqsClient")
      .def(py::init<std::shared_ptr<SqsApi>, std::string, std::vector<std::string>>(), py::arg("api"),
           py::arg("queue_url"), py::arg("attribute_names"))
      .def("num_messages", [](SqsClient& c) {
        Result<int64_t> r;
        {
          py::gil_scoped_release rel;
          r = c.num_messages();
        }
        return unwrap(r);
      })
      .def_property_readonly("queue_url", &SqsClient::queue_url)
      .def_property_readonly("attribute_names", &SqsClient::attribute_names)
      .def_property_readonly("api", &SqsClient::api);

  // ---- Kubernetes ----
  py::class_<ScaleObject>(m, "ScaleObject")
      .def(py::init([](int32_t replicas, bool has_replicas, std::string rv, std::string raw) {
             ScaleObject o;
             o.replicas = replicas;
             o.has_replicas = has_replicas;
             o.resource_version = std::move(rv);
             o.raw = std::move(raw);
             return o;
           }),
           py::arg("replicas") = 0, py::arg("has_replicas") = true, py::arg("resource_version") = "",
           py::arg("raw") = "")
      .def_readwrite("replicas", &ScaleObject::replicas)
      .def_readwrite("has_replicas", &ScaleObject::has_replicas)
      .def_readwrite("resource_version", &ScaleObject::resource_version)
      .def_readwrite("raw", &ScaleObject::raw);
  m.def("parse_scale_object", [](const std::string& j, bool absent_is_zero) {
    return unwrap(parse_scale_object(j, absent_is_zero));
  });

  py::class_<TokenProvider, PyTokenProvider, py::smart_holder>(m, "TokenProvider")
      .def(py::init<>())
      .def("token", [](TokenProvider& t) {
        Result<std::string> r;
        {
          py::gil_scoped_release rel;
          r = t.token();
        }
        return unwrap(r);
      })
      .def("invalidate", [](TokenProvider& t, const std::string& used) { t.invalidate(used); }, py::arg("used"));
  py::class_<StaticTokenProvider, TokenProvider, py::smart_holder>(m, "StaticTokenProvider")
      .def(py::init<std::string>());
  py::class_<FileTokenProvider, TokenProvider, py::smart_holder>(m, "FileTokenProvider")
      .def(py::init<std::string, std::shared_ptr<Clock>, Nanos>(), py::arg("path"), py::arg("clock"),
           py::arg("refresh_ns") = 60 * kSecond);

  py::class_<ExecConfig>(m, "ExecConfig")
      .def(py::init<>())
      .def_readwrite("command", &ExecConfig::command)
      .def_readwrite("args", &ExecConfig::args)
      .def_readwrite("env", &ExecConfig::env)
      .def_readwrite("api_version", &ExecConfig::api_version)
      .def_readwrite("install_hint", &ExecConfig::install_hint)
      .def_readwrite("timeout_ns", &ExecConfig::timeout);
  py::class_<ExecCredential>(m, "ExecCredential")
      .def(py::init<>())
      .def_readonly("token", &ExecCredential::token)
      .def_readonly("cert_pem", &ExecCredential::cert_pem)
      .def_readonly("key_pem", &ExecCredential::key_pem)
      .def_readonly("has_expiry", &ExecCredential::has_expiry)
      .def_readonly("expiry_unix_ns", &ExecCredential::expiry_unix_ns);
  m.def("validate_exec_config", [](const ExecConfig& c) {
    Status s = validate_exec_config(c);
    if (!s.ok()) raise_status(s);
  });
  m.def(
      "run_exec_plugin",
      [](const ExecConfig& c, int code) {
        Result<ExecCredential> r;
        {
          py::gil_scoped_release rel;
          r = run_exec_plugin(c, code);
        }
        return unwrap(r);
      },
      py::arg("config"), py::arg("response_code") = 0);
  py::class_<ExecTokenProvider, TokenProvider, py::smart_holder>(m, "ExecTokenProvider")
      .def(py::init<ExecConfig, std::shared_ptr<Clock>>(), py::arg("config"), py::arg("clock"))
      .def("credential",
           [](ExecTokenProvider& p) {
             Result<ExecCredential> r;
             {
               py::gil_scoped_release rel;
               r = p.credential();
             }
             return unwrap(r);
           })
      .def_property_readonly("runs", &ExecTokenProvider::runs);
  m.def("aws_dns_suffix", &aws_dns_suffix);
  m.def("parse_rfc3339", [](const std::string& s) -> py::object {
    int64_t ns;
    if (!parse_rfc3339(s, &ns)) return py::none();
    return py::int_(ns);
  });

  py::enum_<ScaleMode>(m, "ScaleMode")
      .value("Deployment", ScaleMode::Deployment)
      .value("Scale", ScaleMode::Scale)
      .value("Patch", ScaleMode::Patch);
  py::class_<KubeOptions>(m, "KubeOptions")
      .def(py::init<>())
      .def_readwrite("server", &KubeOptions::server)
      .def_readwrite("namespace", &KubeOptions::namespace_)
      .def_readwrite("mode", &KubeOptions::mode)
      .def_readwrite("tls", &KubeOptions::tls)
      .def_readwrite("token", &KubeOptions::token)
      .def_readwrite("basic_user", &KubeOptions::basic_user)
      .def_readwrite("basic_password", &KubeOptions::basic_password)
      .def_readwrite("timeout_ns", &KubeOptions::timeout)
      .def_readwrite("busy_poll_ns", &KubeOptions::busy_poll)
      .def_readwrite("proxy", &KubeOptions::proxy)
      .def_readwrite("qps", &KubeOptions::qps)
      .def_readwrite("burst", &KubeOptions::burst)
      .def_readwrite("clock", &KubeOptions::clock)
      .def_readwrite("rbac_fallback", &KubeOptions::rbac_fallback)
      .def_readwrite("log", &KubeOptions::log);
  py::class_<TokenBucket>(m, "TokenBucket")
      .def(py::init<double, int, std::shared_ptr<Clock>>(), py::arg("qps"), py::arg("burst"), py::arg("clock"))
      .def("reserve", &TokenBucket::reserve)
      .def("take", [](TokenBucket& b) { return b.take(nullptr); }, py::call_guard<py::gil_scoped_release>());

  py::class_<DeploymentApi, PyDeploymentApi, py::smart_holder>(m, "DeploymentApi")
      .def(py::init<>())
      .def("get", [](DeploymentApi& a, const std::string& name) {
        Result<ScaleObject> r;
        {
          py::gil_scoped_release rel;
          r = a.get(name);
        }
        return unwrap(r);
      })
      .def("update", [](DeploymentApi& a, const std::string& name, const ScaleObject& o, int32_t n) {
        Status s;
        {
          py::gil_scoped_release rel;
          s = a.update(name, o, n);
        }
        if (!s.ok()) raise_status(s);
      });
  py::class_<KubeRestDeployments, DeploymentApi, py::smart_holder>(m, "KubeRestDeployments")
      .def(py::init<KubeOptions>())
      .def("path_for", &KubeRestDeployments::path_for)
      .def_property_readonly("mode", &KubeRestDeployments::mode)
      // the control loop's pipelined read (begin before the SQS call, finish after it)
      .def("set_timing", &KubeRestDeployments::set_timing)
      .def("begin_get", &KubeRestDeployments::begin_get, py::arg("name"), py::arg("may_dial") = true,
           py::call_guard<py::gil_scoped_release>())
      .def("finish_get", [](KubeRestDeployments& k) {
        Result<ScaleObject> r;
        {
          py::gil_scoped_release rel;
          r = k.finish_get();
        }
        return unwrap(r);
      })
      .def("stats", [](KubeRestDeployments& k) {
        auto s = k.stats();
        py::dict d;
        d["gets"] = s.gets;
        d["updates"] = s.updates;
        d["errors"] = s.errors;
        d["conflicts"] = s.conflicts;
        d["throttled"] = s.throttled;
        d["throttle_ns"] = s.throttle_ns;
        d["speculative_skipped"] = s.speculative_skipped;
        d["retry_after"] = s.retry_after;
        d["scale_fallbacks"] = s.scale_fallbacks;
        d["http"] = http_stats_dict(s.http);
        return d;
      });
  py::class_<ScaleSpan>(m, "ScaleSpan")
      .def_readonly("get_ns", &ScaleSpan::get_ns)
      .def_readonly("update_ns", &ScaleSpan::update_ns)
      .def_readonly("read", &ScaleSpan::read)
      .def_readonly("wrote", &ScaleSpan::wrote)
      .def_readonly("before", &ScaleSpan::before)
      .def_readonly("used_prefetch", &ScaleSpan::used_prefetch)
      .def_readonly("refetched", &ScaleSpan::refetched)
      .def_readonly("gets", &ScaleSpan::gets)
      .def_readonly("after", &ScaleSpan::after);

  py::class_<PodAutoScaler, std::shared_ptr<PodAutoScaler>>(m, "PodAutoScaler")
      .def(py::init<std::shared_ptr<DeploymentApi>, std::string, std::string, int64_t, int64_t, int64_t,
                    int64_t, std::shared_ptr<Logger>, std::shared_ptr<Clock>>(),
           py::arg("api"), py::arg("deployment"), py::arg("namespace"), py::arg("max"), py::arg("min"),
           py::arg("scale_up_pods"), py::arg("scale_down_pods"), py::arg("logger"), py::arg("clock"))
      .def("scale_up", [](PodAutoScaler& p) {
        ScaleSpan span;
        Status s;
        {
          py::gil_scoped_release rel;
          s = p.scale_up(&span);
        }
        if (!s.ok()) raise_status(s);
        return span;
      })
      .def_property("dry_run", &PodAutoScaler::dry_run, &PodAutoScaler::set_dry_run)
      .def("prefetch", &PodAutoScaler::prefetch, py::arg("may_dial") = true)
      .def("warm", &PodAutoScaler::warm, py::call_guard<py::gil_scoped_release>())
      .def("discard_prefetch", &PodAutoScaler::discard_prefetch)
      .def("scale_down", [](PodAutoScaler& p) {
        ScaleSpan span;
        Status s;
        {
          py::gil_scoped_release rel;
          s = p.scale_down(&span);
        }
        if (!s.ok()) raise_status(s);
        return span;
      })
      .def_property_readonly("api", &PodAutoScaler::api)
      .def_property_readonly("deployment", &PodAutoScaler::deployment)
      .def_property_readonly("namespace", &PodAutoScaler::namespace_)
      .def_property("max", &PodAutoScaler::max, &PodAutoScaler::set_max)
      .def_property_readonly("min", &PodAutoScaler::min)
      .def_property_readonly("scale_up_pods", &PodAutoScaler::scale_up_pods)
      .def_property_readonly("scale_down_pods", &PodAutoScaler::scale_down_pods);

  // ---- control loop ----
  py::class_<LoopConfig>(m, "LoopConfig")
      .def(py::init<>())
      .def_readwrite("poll_period_ns", &LoopConfig::poll_period)
      .def_readwrite("scale_down_cool_down_ns", &LoopConfig::scale_down_cool_down)
      .def_readwrite("scale_up_cool_down_ns", &LoopConfig::scale_up_cool_down)
      .def_readwrite("scale_up_messages", &LoopConfig::scale_up_messages)
      .def_readwrite("scale_down_messages", &LoopConfig::scale_down_messages)
      .def_readwrite("prefetch", &LoopConfig::prefetch)
      .def_readwrite("prefetch_always", &LoopConfig::prefetch_always)
      .def_readwrite("prewarm_ns", &LoopConfig::prewarm)
      .def_readwrite("presend", &LoopConfig::presend)
      .def_readwrite("prewarm_spin", &LoopConfig::prewarm_spin)
      .def_readwrite("connect_at_start", &LoopConfig::connect_at_start)
      .def_readwrite("spin_budget_ppm", &LoopConfig::spin_budget_ppm);

  py::class_<Runner, std::shared_ptr<Runner>>(m, "Runner")
      .def(py::init<LoopConfig, std::shared_ptr<SqsClient>, std::shared_ptr<PodAutoScaler>, std::shared_ptr<Clock>,
                    std::shared_ptr<Logger>>(),
           py::arg("config"), py::arg("sqs"), py::arg("scaler"), py::arg("clock"), py::arg("logger"))
      .def("arm", &Runner::arm)
      .def("poll_once", [](Runner& r) {
        IterationRecord rec;
        {
          py::gil_scoped_release rel;
          rec = r.poll_once();
        }
        return record_dict(rec);
      })
      .def("step", [](Runner& r) {
        IterationRecord rec;
        {
          py::gil_scoped_release rel;
          rec = r.step(nullptr);
        }
        return record_dict(rec);
      })
      .def("run_iterations", [](Runner& r, int64_t n) {
        py::gil_scoped_release rel;
        r.run(nullptr, n);
      })
      .def("steps", [](Runner& r, int64_t n) {
        std::vector<IterationRecord> recs;
        {
          py::gil_scoped_release rel;
          recs.reserve(static_cast<size_t>(n));
          for (int64_t i = 0; i < n; ++i) recs.push_back(r.step(nullptr));
        }
        py::list out;
        for (auto& rec : recs) out.append(record_dict(rec));
        return out;
      })
      .def("stats", [](Runner& r) {
        auto s = r.stats();
        py::dict d;
        d["polls"] = s.polls;
        d["depth_errors"] = s.depth_errors;
        d["scale_ups"] = s.scale_ups;
        d["scale_downs"] = s.scale_downs;
        d["noop_ups"] = s.noop_ups;
        d["noop_downs"] = s.noop_downs;
        d["cooldown_skips_up"] = s.cooldown_skips_up;
        d["cooldown_skips_down"] = s.cooldown_skips_down;
        d["failed_ups"] = s.failed_ups;
        d["failed_downs"] = s.failed_downs;
        d["speculative_reads"] = s.speculative_reads;
        d["speculative_reads_used"] = s.speculative_reads_used;
        d["speculative_reads_gated"] = s.speculative_reads_gated;
        d["apiserver_reads"] = s.apiserver_reads;
        d["last_depth"] = s.last_depth;
        d["last_replicas"] = s.last_replicas;
        d["latency_samples"] = s.latency_samples;
        d["latency_sum_ns"] = s.latency_sum_ns;
        d["poll_cpu_ns"] = s.poll_cpu_ns;
        d["latency_buckets"] = std::vector<uint64_t>(s.latency_buckets, s.latency_buckets + kLatBuckets);
        d["consecutive_failed_polls"] = s.consecutive_failed_polls;
        return d;
      })
      .def("prewarm_spin_budget", &Runner::prewarm_spin_budget)
      .def("set_spin_budget", &Runner::set_spin_budget)
      .def("idle_ns", &Runner::idle_ns)
      .def("failing_ns", &Runner::failing_ns)
      .def("last_error", &Runner::last_error)
      .def_property("cpus", &Runner::cpus, &Runner::set_cpus)
      .def("set_shared_state", [](Runner& r, uintptr_t addr) {
        r.set_shared_state(addr ? reinterpret_cast<SharedWorkerState*>(addr) : nullptr);
      })
      .def("cancel", &Runner::cancel)
      .def("set_trace_fd", &Runner::set_trace_fd)
      .def("latencies", &Runner::latencies)
      .def("clear_latencies", &Runner::clear_latencies)
      .def_property_readonly("sqs", &Runner::sqs)
      .def_property_readonly("scaler", &Runner::scaler)
      .def_property_readonly("last_scale_up", &Runner::last_scale_up)
      .def_property_readonly("last_scale_down", &Runner::last_scale_down);

  m.attr("latency_bucket_le_ns") = std::vector<int64_t>(kLatBucketLeNs, kLatBucketLeNs + kLatBuckets - 1);

  // ---- process-per-queue fleet: worker state in shared memory (procfleet.py) ----
  auto ws = [](uintptr_t addr) { return reinterpret_cast<SharedWorkerState*>(addr); };
  m.def("shared_worker_state_size", [] { return sizeof(SharedWorkerState); });
  m.def("init_shared_worker_state", [](uintptr_t addr) { init_shared_worker_state(reinterpret_cast<void*>(addr)); });
  m.def("read_shared_worker_state", [ws](uintptr_t addr) {
    SharedWorkerState* s = ws(addr);
    static const char* names[] = {"polls", "depth_errors", "scale_ups", "scale_downs", "noop_ups", "noop_downs",
                                  "cooldown_skips_up", "cooldown_skips_down", "failed_ups", "failed_downs",
                                  "speculative_reads", "speculative_reads_used", "speculative_reads_gated",
                                  "apiserver_reads", "latency_samples", "consecutive_failed_polls", "poll_cpu_ns"};
    static_assert(sizeof(names) / sizeof(names[0]) == SharedWorkerState::kNumCounters, "counter names");
    py::dict d;
    for (int i = 0; i < SharedWorkerState::kNumCounters; ++i)
      d[names[i]] = s->counters[i].load(std::memory_order_acquire);
    d["progress_ns"] = s->progress_ns.load(std::memory_order_acquire);
    d["last_good_ns"] = s->last_good_ns.load(std::memory_order_relaxed);
    d["last_depth"] = s->last_depth.load(std::memory_order_relaxed);
    d["last_replicas"] = s->last_replicas.load(std::memory_order_relaxed);
    d["latency_sum_ns"] = s->lat_sum_ns.load(std::memory_order_relaxed);
    std::vector<uint64_t> hist(kLatBuckets);
    for (int i = 0; i < kLatBuckets; ++i) hist[i] = s->lat_hist[i].load(std::memory_order_relaxed);
    d["latency_buckets"] = hist;
    d["status"] = s->status.load(std::memory_order_acquire);
    d["control"] = s->control.load(std::memory_order_acquire);
    d["max_override"] = s->max_override.load(std::memory_order_relaxed);
    d["iterations"] = s->iterations.load(std::memory_order_relaxed);
    return d;
  });
  m.def("read_shared_worker_error", [ws](uintptr_t addr) {
    const std::string t = read_shared_error(ws(addr));
    return py::reinterpret_steal<py::str>(PyUnicode_DecodeUTF8(t.data(), static_cast<Py_ssize_t>(t.size()), "replace"));
  });
  m.def("write_shared_worker_error", [ws](uintptr_t addr, const std::string& t) { write_shared_error(ws(addr), t); });
  m.def("shared_worker_latencies", [ws](uintptr_t addr) {
    SharedWorkerState* s = ws(addr);
    const uint64_t n = s->counters[SharedWorkerState::kLatencySamples].load(std::memory_order_acquire);
    const uint64_t keep = std::min<uint64_t>(n, SharedWorkerState::kRing);
    std::vector<int64_t> out;
    out.reserve(keep);
    for (uint64_t i = n - keep; i < n; ++i)
      out.push_back(s->lat_ring[i % SharedWorkerState::kRing].load(std::memory_order_relaxed));
    return out;
  });
  m.def("set_shared_worker_control", [ws](uintptr_t addr, int32_t c) { ws(addr)->control.store(c, std::memory_order_release); });
  m.def("set_shared_worker_status", [ws](uintptr_t addr, int32_t c) { ws(addr)->status.store(c, std::memory_order_release); });
  m.def("set_shared_worker_max", [ws](uintptr_t addr, int64_t v) { ws(addr)->max_override.store(v, std::memory_order_relaxed); });
  m.def("set_shared_worker_iterations", [ws](uintptr_t addr, int64_t v) { ws(addr)->iterations.store(v, std::memory_order_relaxed); });
  m.def("set_shared_worker_progress", [ws](uintptr_t addr, int64_t v) { ws(addr)->progress_ns.store(v, std::memory_order_release); });

  py::class_<Supervisor, std::shared_ptr<Supervisor>>(m, "Supervisor")
      .def(py::init<>())
      .def("add", &Supervisor::add)
      .def_property("stagger", &Supervisor::stagger, &Supervisor::set_stagger)
      // start may wait for a runner's HomeThread to finish a previous run (whose observer may
      // need the GIL)
      .def("start", &Supervisor::start, py::arg("max_iterations") = -1, py::call_guard<py::gil_scoped_release>())
      .def("stop", &Supervisor::stop)
      .def("stopped", &Supervisor::stopped)
      .def("wait", &Supervisor::wait, py::arg("timeout_ns"), py::call_guard<py::gil_scoped_release>())
      .def("join", &Supervisor::join, py::call_guard<py::gil_scoped_release>())
      .def("__len__", &Supervisor::size)
      .def("runner", &Supervisor::runner)
      .def("thread_sched", [](Supervisor& s) {
        auto t = s.thread_sched();
        py::dict d;
        d["threads"] = t.threads;
        d["cpu_ns"] = t.cpu_ns;
        d["runq_wait_ns"] = t.runq_wait_ns;
        d["slices"] = t.slices;
        d["vol_cs"] = t.vol_cs;
        d["invol_cs"] = t.invol_cs;
        d["utime_ns"] = t.utime_ns;
        d["stime_ns"] = t.stime_ns;
        d["minflt"] = t.minflt;
        return d;
      });

  py::class_<Scheduler, std::shared_ptr<Scheduler>>(m, "Scheduler")
      .def(py::init([](size_t threads, bool stagger) {
             return std::make_shared<Scheduler>(threads, std::make_shared<RealClock>(), stagger);
           }),
           py::arg("threads"), py::arg("stagger") = true)
      .def("reset_lateness", &Scheduler::reset_lateness)
      .def("add", &Scheduler::add)
      .def("start", &Scheduler::start, py::arg("max_iterations") = -1)
      .def("stop", &Scheduler::stop)
      .def("stopped", &Scheduler::stopped)
      .def("wait", &Scheduler::wait, py::arg("timeout_ns"), py::call_guard<py::gil_scoped_release>())
      .def("join", &Scheduler::join, py::call_guard<py::gil_scoped_release>())
      .def("__len__", &Scheduler::size)
      .def("threads", &Scheduler::threads)
      .def("runner", &Scheduler::runner)
      .def("late_polls", &Scheduler::late_polls)
      .def("max_lateness_ns", &Scheduler::max_lateness);

  m.def("percentile", &percentile);

  // ---- what-if policy sweep (CPU path; the gfx950 kernel is in libksa_gpu.so) ----
  using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;
  using I32 = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;
  m.def("sweep_cpu",
        [](I64 trace_t, I64 trace_d, int32_t init, int64_t horizon, I64 latency, I64 params, int threads, bool ns_clock,
           int skip) {
          if (trace_t.ndim() != 1 || trace_d.ndim() != 1 || trace_t.shape(0) != trace_d.shape(0) || trace_t.shape(0) < 1)
            throw py::value_error("trace_t / trace_d must be 1-D arrays of equal non-zero length");
          if (trace_t.at(0) != 0) throw py::value_error("the trace must start at t=0");
          if (latency.size() != 3) throw py::value_error("latency must be (sqs, get, update) ns");
          if (params.ndim() != 2 || params.shape(0) != 9) throw py::value_error("params must have shape (9, m)");
          const int64_t m = params.shape(1);
          I64 out64({int64_t(3), m});
          I32 out32({int64_t(7), m});
          if (skip < 0 || skip > 2) throw py::value_error("skip must be 0 (auto), 1 (always) or 2 (never)");
          int used = 0;
          {
            py::gil_scoped_release rel;
            used = sweep_cpu(trace_t.data(), trace_d.data(), static_cast<int32_t>(trace_t.shape(0)), init, horizon,
                             latency.data(), params.data(), m, out64.mutable_data(), out32.mutable_data(), threads,
                             (ns_clock ? 1 : 0) | (skip << 2));
          }
          return py::make_tuple(out64, out32, (used & 1) != 0, (used & 2) != 0);
        },
        py::arg("trace_t"), py::arg("trace_d"), py::arg("init_replicas"), py::arg("horizon_ns"), py::arg("latency"),
        py::arg("params"), py::arg("threads") = 8, py::arg("ns_clock") = false, py::arg("skip") = 0);

  m.def("queue_sweep_cpu",
        [](I64 t_ms, I64 rate_milli, int32_t init, int64_t horizon, I64 latency, I64 model, I64 params, int32_t seeds,
           uint64_t seed0, int threads, int arith) {
          if (t_ms.ndim() != 1 || rate_milli.ndim() != 1 || t_ms.shape(0) != rate_milli.shape(0) || t_ms.shape(0) < 1)
            throw py::value_error("t_ms / rate_milli must be 1-D arrays of equal non-zero length");
          if (t_ms.at(0) != 0) throw py::value_error("the arrival trace must start at t=0");
          if (latency.size() != 3) throw py::value_error("latency must be (sqs, get, update) ns");
          if (model.size() != 4) throw py::value_error("model must be (service_milli, startup_ns, slo_backlog, init_backlog)");
          if (params.ndim() != 2 || params.shape(0) != 9) throw py::value_error("params must have shape (9, m)");
          if (seeds < 1) throw py::value_error("seeds must be >= 1");
          const int64_t lanes = params.shape(1) * seeds;
          I64 out64({int64_t(7), lanes});
          I32 out32({int64_t(5), lanes});
          int used = 0;
          {
            py::gil_scoped_release rel;
            used = queue_sweep_cpu(t_ms.data(), rate_milli.data(), static_cast<int32_t>(t_ms.shape(0)), init, horizon,
                                   latency.data(), model.data(), params.data(), params.shape(1), seeds, seed0,
                                   out64.mutable_data(), out32.mutable_data(), threads, arith);
          }
          return py::make_tuple(out64, out32, (used & 1) != 0, (used & 2) != 0);
        },
        py::arg("t_ms"), py::arg("rate_milli"), py::arg("init_replicas"), py::arg("horizon_ns"), py::arg("latency"),
        py::arg("model"), py::arg("params"), py::arg("seeds"), py::arg("seed0") = 1, py::arg("threads") = 8,
        py::arg("arith") = 0);

  m.attr("HTTP_TIMING") = kHttpTiming;  // false in the image build (-DKSA_HTTP_TIMING=0)
  m.attr("HTTP_MAX_SPIN_THROUGH_NS") = HttpClient::kMaxSpinThrough;
  m.attr("SECOND") = kSecond;
  m.attr("MILLISECOND") = kMillisecond;
  m.attr("MICROSECOND") = kMicrosecond;
}
