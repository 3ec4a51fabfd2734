# One GPU-box pass: build, GPU tests, smoke, bench, rocprof of the GPU kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-sweep > gpurun_out/bench_steps20.json 2> gpurun_out/bench_steps20.err &&
timeout -k 10 300 python bench.py --queues 8 --no-sweep > gpurun_out/bench_q8.json 2> gpurun_out/bench_q8.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o sweep -- python3 scripts/sweep_bench.py > gpurun_out/prof_sweep.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o queue -- python3 scripts/queue_sweep_bench.py > gpurun_out/prof_queue.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
