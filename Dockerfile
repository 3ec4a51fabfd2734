# Two stages like the reference (/root/reference/Dockerfile): build the native runtime, then ship a
# runtime image. Targets:
#   runtime (default) -- ROCm base; includes libksa_gpu.so for --gpu-aware-max=local, which runs the
#                        gfx950 HBM probe when the autoscaler is a sidecar on the MI355X node.
#   slim              -- plain Ubuntu + Python + OpenSSL, no GPU code: the control loop alone needs
#                        none (docker build --target slim).
# Both put the launcher at /kube-sqs-autoscaler, so the reference's manifests
# (`command: [/kube-sqs-autoscaler, --flags...]`, README.md:37-39) work unchanged.
FROM rocm/dev-ubuntu-22.04:7.2 AS builder
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-pip g++ libssl-dev \
 && rm -rf /var/lib/apt/lists/*
WORKDIR /work
COPY . /work
RUN pip3 install --no-cache-dir pybind11 PyYAML prometheus-client \
 && PYTORCH_ROCM_ARCH=gfx950 python3 -m kube_sqs_autoscaler_amd.ops.build

FROM ubuntu:22.04 AS slim
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-pip ca-certificates libssl3 \
 && rm -rf /var/lib/apt/lists/* && pip3 install --no-cache-dir PyYAML prometheus-client
COPY --from=builder /work/kube_sqs_autoscaler_amd /app/kube_sqs_autoscaler_amd
COPY --from=builder /work/deploy/bin/kube-sqs-autoscaler /kube-sqs-autoscaler
RUN rm -f /app/kube_sqs_autoscaler_amd/ops/libksa_gpu.so /app/kube_sqs_autoscaler_amd/ops/*.bin
ENV PYTHONPATH=/app KSA_NO_AUTOBUILD=1
USER 65534
ENTRYPOINT ["/kube-sqs-autoscaler"]

FROM rocm/dev-ubuntu-22.04:7.2 AS runtime
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-pip ca-certificates libssl3 \
 && rm -rf /var/lib/apt/lists/* && pip3 install --no-cache-dir PyYAML prometheus-client
COPY --from=builder /work/kube_sqs_autoscaler_amd /app/kube_sqs_autoscaler_amd
COPY --from=builder /work/deploy/bin/kube-sqs-autoscaler /kube-sqs-autoscaler
ENV PYTHONPATH=/app KSA_NO_AUTOBUILD=1
USER 65534
ENTRYPOINT ["/kube-sqs-autoscaler"]
