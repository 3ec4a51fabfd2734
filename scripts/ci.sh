#!/usr/bin/env bash
# CI gate (the reference ran `make test` on Travis, .travis.yml): native build incl. the gfx950
# cross-compile, host C++ tests plain/ASan+UBSan/TSan, a minute of wire-parser fuzzing, then the
# CPU Python suite.
set -euo pipefail
cd "$(dirname "$0")/.."
python3 -m kube_sqs_autoscaler_amd.ops.build --sanitizers
./build/native_tests
./build/native_tests_asan
TSAN_OPTIONS="halt_on_error=1" ./build/native_tests_tsan
python3 -m kube_sqs_autoscaler_amd.ops.build --no-hip --fuzz
mkdir -p build/fuzz_corpus && ./build/fuzz_wire -max_total_time=60 -timeout=10 build/fuzz_corpus csrc/tests/fuzz_corpus
# parallel over the runner's CPUs (pytest-xdist); the timing-sensitive `serial` tests skip
# themselves under xdist workers and run afterwards on their own
python3 -m pytest tests -q -m "not gpu" -n auto
python3 -m pytest tests -q -m "serial and not gpu"
