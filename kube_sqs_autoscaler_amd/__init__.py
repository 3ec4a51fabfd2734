"""kube_sqs_autoscaler_amd -- an SQS-queue-depth autoscaler for GPU-worker Deployments on MI355X nodes.

Capabilities match AcceleratorApp/kube-sqs-autoscaler (same CLI flags, cool-down semantics and
Deployment scaling behaviour); the runtime is native C++ (``csrc/``) behind pybind11 bindings.

Layout:
  config.py        Go-flag CLI surface + configuration model          (reference main.go)
  autoscaler.py    factories: config -> native SQS/kube clients/loop  (sqs/sqs.go, scale/scale.go)
  cli.py           process entry point                               (main.go:82-116)
  models/          decision model: reference oracle, traces, parity  (main.go:35-80 semantics)
  ops/             native runtime loader, build, gfx950 probe
  parallel/        multi-queue worker fleet
  sqs/, kube/      AWS credential chain, kube config loading
  bench/           poll->patch latency benchmark
  metrics.py       Prometheus + health endpoints
"""
__version__ = "0.1.0"
