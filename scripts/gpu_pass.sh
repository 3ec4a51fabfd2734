# GPU-box pass on the tree as built in the container (no rebuild, as the driver runs it):
# GPU tests, smoke, headline bench, the driver's 20-step form and the 8-queue timed run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-sweep > gpurun_out/bench_steps20.json 2> gpurun_out/bench_steps20.err &&
timeout -k 10 300 python bench.py --queues 8 --no-sweep > gpurun_out/bench_q8.json 2> gpurun_out/bench_q8.err
rc=$?
echo "exit $rc"
exit $rc
