set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "sweep or closed" > gpurun_out/ab_pytest.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o sweep -- python3 scripts/sweep_bench.py > gpurun_out/ab_sweep.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o queue -- python3 scripts/queue_sweep_bench.py > gpurun_out/ab_queue.log 2>&1
