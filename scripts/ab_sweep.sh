# Sweep-kernel A/B on one GPU box: the 1M-configuration bench (scripts/sweep_bench.py) with the
# in-tree library and with alternative builds passed as arguments (KSA_GPU_LIB), alternating over
# two rounds; then the exactness test. Results in gpurun_out/ab/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for round in 1 2; do
  timeout -k 10 120 python scripts/sweep_bench.py > gpurun_out/ab/intree_$round.jsonl 2>&1 || exit 1
  for lib in "$@"; do
    KSA_GPU_LIB=$PWD/$lib timeout -k 10 120 python scripts/sweep_bench.py > gpurun_out/ab/$(basename $lib .so)_$round.jsonl 2>&1 || exit 1
  done
done
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k sweep > gpurun_out/ab/pytest.log 2>&1
