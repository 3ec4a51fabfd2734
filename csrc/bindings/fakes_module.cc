// Python bindings for the native test doubles (`kube_sqs_autoscaler_amd.ops._ksa_fakes`): the
// localhost fake SQS / kube-apiserver endpoints (csrc/fakes/fakes.h), their HTTP server, and the
// in-process fakes of the two API seams (csrc/fakes/mem_fakes.h) -- the reference's MockSQS
// (/root/reference/sqs/sqs_test.go:27-59) and fake clientset (/root/reference/scale/scale_test.go:85-115).
//
// Tests, the benchmark and the decision-parity harness load this module next to _ksa_native; the
// production image ships only _ksa_native. Classes derive from the seams _ksa_native registers
// (SqsApi, DeploymentApi), so this module imports it first and a MockSqsApi plugs into a native
// Runner like any SqsApi; errors raise _ksa_native.NativeError.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../core/clock.h"
#include "../fakes/fakes.h"
#include "../fakes/http_server.h"
#include "../fakes/mem_fakes.h"

namespace py = pybind11;
using namespace ksa;

namespace {

py::object g_native_error;  // kube_sqs_autoscaler_amd.ops._ksa_native.NativeError

[[noreturn]] void raise_status(const Status& s) {
  PyErr_SetString(g_native_error.ptr(), s.message().c_str());
  throw py::error_already_set();
}

}  // namespace

PYBIND11_MODULE(_ksa_fakes, m) {
  m.doc() = "Native test doubles of the MI355X SQS autoscaler (fake endpoints, in-memory API fakes).";
  py::module_ native = py::module_::import("kube_sqs_autoscaler_amd.ops._ksa_native");
  g_native_error = native.attr("NativeError");
  m.attr("NativeError") = g_native_error;

  m.def("generate_self_signed", [](const std::string& host) {
    std::string c, k;
    Status s = generate_self_signed(host, &c, &k);
    if (!s.ok()) raise_status(s);
    return py::make_tuple(c, k);
  });


  // ---- in-memory fakes of the API seams ----
  py::class_<MockSqsApi, SqsApi, py::smart_holder>(m, "MockSqsApi")
      .def(py::init<AttrMap>(), py::arg("attributes") = AttrMap{})
      .def("set_attributes", &MockSqsApi::set_attributes)
      .def("set_latency", &MockSqsApi::set_latency)
      .def("fail_next", &MockSqsApi::fail_next)
      .def("calls", &MockSqsApi::calls);
  py::class_<TraceSqsApi, SqsApi, py::smart_holder>(m, "TraceSqsApi")
      .def(py::init<std::shared_ptr<Clock>, std::vector<std::pair<Nanos, AttrMap>>, Nanos>(),
           py::arg("clock"), py::arg("segments"), py::arg("per_call_latency_ns") = 0);
  py::class_<FakeDeployments, DeploymentApi, py::smart_holder>(m, "FakeDeployments")
      .def(py::init<std::string>(), py::arg("namespace") = "namespace")
      .def("add", &FakeDeployments::add)
      .def("add_without_replicas", &FakeDeployments::add_without_replicas)
      .def("replicas", &FakeDeployments::replicas)
      .def("set_replicas", &FakeDeployments::set_replicas)
      .def("set_latency", &FakeDeployments::set_latency)
      .def("fail_next_get", &FakeDeployments::fail_next_get)
      .def("fail_next_update", &FakeDeployments::fail_next_update)
      .def("conflict_next", &FakeDeployments::conflict_next)
      .def("enable_pipelining", &FakeDeployments::enable_pipelining)
      .def("gets", &FakeDeployments::gets)
      .def("updates", &FakeDeployments::updates);


  // ---- fakes ----
  py::class_<InjectedFault>(m, "InjectedFault")
      .def(py::init([](int status, std::string body, std::string ct, bool drop, std::string retry_after,
                       std::string method) {
             InjectedFault f;
             f.status = status;
             f.body = std::move(body);
             f.content_type = std::move(ct);
             f.drop_connection = drop;
             f.retry_after = std::move(retry_after);
             f.method = std::move(method);
             return f;
           }),
           py::arg("status") = 500, py::arg("body") = "", py::arg("content_type") = "text/plain",
           py::arg("drop_connection") = false, py::arg("retry_after") = "", py::arg("method") = "");

  py::class_<FakeSqsServer, std::shared_ptr<FakeSqsServer>>(m, "FakeSqsServer")
      .def(py::init<>())
      .def("require_signature", &FakeSqsServer::require_signature)
      .def("start",
           [](FakeSqsServer& s, const std::string& host, int port, bool tls) {
             Status st = s.start(host, port, tls);
             if (!st.ok()) raise_status(st);
           },
           py::arg("host") = "127.0.0.1", py::arg("port") = 0, py::arg("tls") = false)
      .def("stop", &FakeSqsServer::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &FakeSqsServer::port)
      .def_property_readonly("url", &FakeSqsServer::url)
      .def_property_readonly("cert_pem", &FakeSqsServer::cert_pem)
      .def("set_attributes", &FakeSqsServer::set_attributes)
      .def("set_default_attributes", &FakeSqsServer::set_default_attributes)
      .def("set_attribute_cycle", &FakeSqsServer::set_attribute_cycle)
      .def("inject", &FakeSqsServer::inject)
      .def("set_latency", &FakeSqsServer::set_latency)
      .def("set_cpus", &FakeSqsServer::set_cpus)
      .def("set_hot", &FakeSqsServer::set_hot)
      .def("set_timing", &FakeSqsServer::set_timing)
      .def("drop_connections", &FakeSqsServer::drop_connections)
      .def("requests", &FakeSqsServer::requests)
      .def("signature_failures", &FakeSqsServer::signature_failures)
      .def("connections", &FakeSqsServer::connections)
      .def("connection_threads", &FakeSqsServer::connection_threads)
      .def("timings", [](const FakeSqsServer& s) {
        std::vector<std::pair<int64_t, int64_t>> out;
        for (auto& t : s.timings()) out.emplace_back(t.wake_ns, t.service_ns);
        return out;
      })
      .def("clear_timings", &FakeSqsServer::clear_timings)
      .def("last_body", &FakeSqsServer::last_body)
      .def("last_headers", &FakeSqsServer::last_headers);

  py::class_<FakeKubeServer, std::shared_ptr<FakeKubeServer>>(m, "FakeKubeServer")
      .def(py::init<>())
      .def("require_token", &FakeKubeServer::require_token)
      .def("start",
           [](FakeKubeServer& s, const std::string& host, int port, bool tls) {
             Status st = s.start(host, port, tls);
             if (!st.ok()) raise_status(st);
           },
           py::arg("host") = "127.0.0.1", py::arg("port") = 0, py::arg("tls") = false)
      .def("stop", &FakeKubeServer::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &FakeKubeServer::port)
      .def_property_readonly("url", &FakeKubeServer::url)
      .def_property_readonly("cert_pem", &FakeKubeServer::cert_pem)
      .def("add_deployment", &FakeKubeServer::add_deployment)
      .def("replicas", &FakeKubeServer::replicas)
      .def("set_replicas", &FakeKubeServer::set_replicas)
      .def("deployment_json", &FakeKubeServer::deployment_json)
      .def("lease_json", &FakeKubeServer::lease_json)
      .def("add_node", &FakeKubeServer::add_node, py::arg("name"), py::arg("labels"), py::arg("resource"),
           py::arg("gpus"), py::arg("unschedulable") = false)
      .def("inject", &FakeKubeServer::inject)
      .def("conflict_next", &FakeKubeServer::conflict_next)
      .def("set_rbac", &FakeKubeServer::set_rbac)
      .def("forbidden", &FakeKubeServer::forbidden)
      .def("set_latency", &FakeKubeServer::set_latency)
      .def("set_cpus", &FakeKubeServer::set_cpus)
      .def("set_hot", &FakeKubeServer::set_hot)
      .def("set_timing", &FakeKubeServer::set_timing)
      .def("drop_connections", &FakeKubeServer::drop_connections)
      .def("requests", &FakeKubeServer::requests)
      .def("gets", &FakeKubeServer::gets)
      .def("writes", &FakeKubeServer::writes)
      .def("conflicts", &FakeKubeServer::conflicts)
      .def("auth_failures", &FakeKubeServer::auth_failures)
      .def("connections", &FakeKubeServer::connections)
      .def("timings", [](const FakeKubeServer& s) {
        std::vector<std::pair<int64_t, int64_t>> out;
        for (auto& t : s.timings()) out.emplace_back(t.wake_ns, t.service_ns);
        return out;
      })
      .def("clear_timings", &FakeKubeServer::clear_timings)
      .def("last_method", &FakeKubeServer::last_method)
      .def("last_body", &FakeKubeServer::last_body)
      .def("last_path", &FakeKubeServer::last_path);

}
