# The headline detail probe in 8 fresh processes: run-to-run spread of p50 and phases.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 120 python -u scripts/headline_detail.py >> gpurun_out/repeat_detail.jsonl 2>> gpurun_out/repeat.err || exit 1
done
