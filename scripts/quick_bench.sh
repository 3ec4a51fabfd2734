# Headline only, three back-to-back runs (no secondary sweep), then the per-phase detail probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-sweep >> gpurun_out/quick_bench.jsonl 2>> gpurun_out/quick_bench.err || exit 1
done
timeout -k 10 200 python -u scripts/headline_detail.py > gpurun_out/quick_detail.jsonl 2>> gpurun_out/quick_bench.err
