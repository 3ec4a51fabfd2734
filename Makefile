# Mirrors the reference Makefile targets (test / compile / build / push) for this build.
.PHONY: test test-gpu compile native sanitize fuzz ci bench build push clean

IMAGE ?= kube-sqs-autoscaler-amd
VERSION ?= v0.1.0
PY ?= python3

test:            ## CPU test suite (no GPU needed): parallel, then the timing-sensitive tests serially
	$(PY) -m pytest tests -q -m "not gpu" -n auto
	$(PY) -m pytest tests -q -m "serial and not gpu"

test-gpu:        ## GPU tests on an MI355X box
	$(PY) -m pytest tests -q -m gpu

compile native:  ## native runtime + gfx950 probe, in-tree
	$(PY) -m kube_sqs_autoscaler_amd.ops.build

sanitize:        ## host C++ unit tests under ASan/UBSan and TSan
	$(PY) -m kube_sqs_autoscaler_amd.ops.build --no-hip --sanitizers
	./build/native_tests && ./build/native_tests_asan && ./build/native_tests_tsan

fuzz:            ## libFuzzer + ASan/UBSan over the wire parsers (10 minutes)
	$(PY) -m kube_sqs_autoscaler_amd.ops.build --no-hip --fuzz
	mkdir -p build/fuzz_corpus && ./build/fuzz_wire -max_total_time=600 -timeout=10 build/fuzz_corpus csrc/tests/fuzz_corpus

ci:              ## what CI runs (no network, no package installs)
	bash scripts/ci.sh

bench:
	$(PY) bench.py

build:
	docker build -t $(IMAGE):$(VERSION) .

push: build
	docker push $(IMAGE):$(VERSION)

clean:
	rm -rf build kube_sqs_autoscaler_amd/ops/*.so
