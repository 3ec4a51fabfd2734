# Sweep-kernel A/B on one GPU box: a sweep bench ($BENCH, default the 1M-configuration
# scripts/sweep_bench.py; scripts/queue_sweep_bench.py for the closed loop) with the in-tree library and with alternative builds passed as arguments (KSA_GPU_LIB), alternating over
# two rounds; then the exactness test. Results in gpurun_out/ab/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
BENCH=${BENCH:-scripts/sweep_bench.py}
tag=$(basename $BENCH .py)
for round in 1 2; do
  timeout -k 10 120 python $BENCH > gpurun_out/ab/${tag}_intree_$round.jsonl 2>&1 || exit 1
  for lib in "$@"; do
    KSA_GPU_LIB=$PWD/$lib timeout -k 10 120 python $BENCH > gpurun_out/ab/${tag}_$(basename $lib .so)_$round.jsonl 2>&1 || exit 1
  done
done
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k sweep > gpurun_out/ab/pytest.log 2>&1
