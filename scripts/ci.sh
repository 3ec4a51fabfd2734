#!/usr/bin/env bash
# CI gate (the reference ran `make test` on Travis, .travis.yml): native build incl. the gfx950
# cross-compile, host C++ tests plain/ASan+UBSan/TSan, then the CPU Python suite.
set -euo pipefail
cd "$(dirname "$0")/.."
python3 -m kube_sqs_autoscaler_amd.ops.build --sanitizers
./build/native_tests
./build/native_tests_asan
TSAN_OPTIONS="halt_on_error=1" ./build/native_tests_tsan
python3 -m pytest tests -q -m "not gpu"
