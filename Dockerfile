# Build, then a small runtime image, like the reference (/root/reference/Dockerfile:1-9).
# Targets (the LAST stage is what a plain `docker build .` produces):
#   slim  -- (default) Ubuntu + Python + OpenSSL, no GPU code: the control loop needs none. Built
#            by `slim-builder` from plain ubuntu:22.04 (g++, libssl-dev, pybind11): no ROCm
#            anywhere in its stage chain (tests/test_image_layout.py checks this).
#   gpu   -- adds the HIP *runtime* (hip-runtime-amd from the ROCm apt repository, no compiler or
#            dev packages) and libksa_gpu.so, for --gpu-aware-max=local: the gfx950 HBM probe of a
#            sidecar on the MI355X node (docker build --target gpu). Built by `gpu-builder`, the
#            ROCm toolchain image (hipcc --offload-arch=gfx950).
# Both builders run the native C++ tests, then `ops.build --image`: _ksa_native with the HTTP
# timing diagnostics compiled out and the test doubles (_ksa_fakes) removed from the package.
# Both images put the launcher at /kube-sqs-autoscaler, so the reference's manifests
# (`command: [/kube-sqs-autoscaler, --flags...]`, README.md:37-39) work unchanged, and with the
# /scale -> Deployment fallback so does a Role written for the reference (get/update deployments).
ARG ROCM_VERSION=7.2

FROM ubuntu:22.04 AS slim-builder
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-pip g++ libssl-dev \
 && rm -rf /var/lib/apt/lists/*
WORKDIR /work
COPY . /work
# pybind11 3 (smart_holder) is not in Ubuntu 22.04's archive: pinned from PyPI, build stage only.
RUN pip3 install --no-cache-dir pybind11==3.0.4 \
 && python3 -m kube_sqs_autoscaler_amd.ops.build --no-hip --sanitizers \
 && ./build/native_tests \
 && python3 -m kube_sqs_autoscaler_amd.ops.build --no-hip --image

FROM rocm/dev-ubuntu-22.04:${ROCM_VERSION} AS gpu-builder
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-pip g++ libssl-dev \
 && rm -rf /var/lib/apt/lists/*
WORKDIR /work
COPY . /work
RUN pip3 install --no-cache-dir pybind11==3.0.4 \
 && python3 -m kube_sqs_autoscaler_amd.ops.build --no-hip --sanitizers \
 && ./build/native_tests \
 && PYTORCH_ROCM_ARCH=gfx950 python3 -m kube_sqs_autoscaler_amd.ops.build --image

FROM ubuntu:22.04 AS runtime
# Runtime Python deps from the distribution archive (no pip at runtime).
RUN apt-get update && apt-get install -y --no-install-recommends python3 python3-yaml ca-certificates libssl3 \
 && rm -rf /var/lib/apt/lists/*
COPY deploy/bin/kube-sqs-autoscaler /kube-sqs-autoscaler
ENV PYTHONPATH=/app KSA_NO_AUTOBUILD=1

FROM runtime AS gpu
ARG ROCM_VERSION
RUN apt-get update && apt-get install -y --no-install-recommends curl gnupg \
 && mkdir -p /etc/apt/keyrings \
 && curl -fsSL https://repo.radeon.com/rocm/rocm.gpg.key | gpg --dearmor -o /etc/apt/keyrings/rocm.gpg \
 && echo "deb [arch=amd64 signed-by=/etc/apt/keyrings/rocm.gpg] https://repo.radeon.com/rocm/apt/${ROCM_VERSION} jammy main" \
      > /etc/apt/sources.list.d/rocm.list \
 && apt-get update && apt-get install -y --no-install-recommends hip-runtime-amd \
 && apt-get purge -y curl gnupg && apt-get autoremove -y && rm -rf /var/lib/apt/lists/*
COPY --from=gpu-builder /work/kube_sqs_autoscaler_amd /app/kube_sqs_autoscaler_amd
ENV LD_LIBRARY_PATH=/opt/rocm/lib
USER 65534
ENTRYPOINT ["/kube-sqs-autoscaler"]

FROM runtime AS slim
COPY --from=slim-builder /work/kube_sqs_autoscaler_amd /app/kube_sqs_autoscaler_amd
USER 65534
ENTRYPOINT ["/kube-sqs-autoscaler"]
