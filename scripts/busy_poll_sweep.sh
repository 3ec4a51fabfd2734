# Busy-poll window sweep on the GPU box host (1 and 8 queues), one JSON line per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for q in 1 8; do
  for bp in 0 25 50 100 200; do
    timeout -k 10 120 python bench.py --queues $q --steps 3000 --warmup 300 --no-sweep --busy-poll-us $bp >> gpurun_out/busy_poll_sweep.jsonl 2>> gpurun_out/busy_poll_sweep.err || exit 1
  done
done
echo done
