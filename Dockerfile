# Two stages like the reference (/root/reference/Dockerfile): build the native runtime, then ship a
# runtime image. The autoscaler itself needs no GPU; the ROCm base is only required for the
# optional --gpu-aware-max probe (libksa_gpu.so) when it runs as a sidecar on the MI355X node.
FROM rocm/dev-ubuntu-22.04:7.2 AS builder
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-pip g++ libssl-dev \
 && rm -rf /var/lib/apt/lists/*
WORKDIR /work
COPY . /work
RUN pip3 install --no-cache-dir pybind11 PyYAML prometheus-client \
 && PYTORCH_ROCM_ARCH=gfx950 python3 -m kube_sqs_autoscaler_amd.ops.build

FROM rocm/dev-ubuntu-22.04:7.2
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-pip ca-certificates libssl3 \
 && rm -rf /var/lib/apt/lists/* && pip3 install --no-cache-dir pybind11 PyYAML prometheus-client
COPY --from=builder /work/kube_sqs_autoscaler_amd /app/kube_sqs_autoscaler_amd
ENV PYTHONPATH=/app KSA_NO_AUTOBUILD=1
USER 65534
ENTRYPOINT ["python3", "-m", "kube_sqs_autoscaler_amd"]
