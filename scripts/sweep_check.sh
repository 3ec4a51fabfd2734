# Sweep kernel: GPU tests + profiled throughput run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 &&
timeout -k 10 300 python -m pytest tests/test_gpu.py -x -q -k sweep > gpurun_out/pytest_sweep.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o sweep -- python3 scripts/sweep_bench.py > gpurun_out/prof_sweep.log 2>&1
