# One GPU-box pass: build, GPU tests, smoke, bench, the sharding and 5 s cadence evidence, and
# rocprofv3 of the GPU kernels. Every step has its own time limit; the first failure ends the pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 --no-sweep --rehearse-shared-gpus > gpurun_out/bench_ranks2.json 2> gpurun_out/bench_ranks2.err &&
timeout -k 10 300 python scripts/shard_balance.py --world 8 > gpurun_out/shard_balance.jsonl 2> gpurun_out/shard_balance.err &&
timeout -k 10 300 python scripts/cadence_5s.py > gpurun_out/cadence_5s.jsonl 2> gpurun_out/cadence_5s.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o sweep -- python3 scripts/sweep_bench.py > gpurun_out/prof_sweep.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o queue -- python3 scripts/queue_sweep_bench.py > gpurun_out/prof_queue.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
