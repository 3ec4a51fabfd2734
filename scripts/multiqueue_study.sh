# The r02 multi-queue study in one call (profiles/README.md "r02: multi-queue"): scheduler view
# per thread group, explicit placements, threads vs processes at a fixed placement, a bare TCP
# loopback echo, and --worker-processes vs threads. Results: gpurun_out/mq_study/*.jsonl
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/mq_study
mkdir -p $out
timeout -k 10 300 python scripts/multiqueue_probe.py --servers shared per-queue processes > $out/sched.jsonl 2> $out/sched.err &&
timeout -k 10 300 python scripts/placement_probe.py --layouts none ccd smt sockets > $out/placement.jsonl 2> $out/placement.err &&
timeout -k 10 300 python scripts/ranks_probe.py > $out/ranks.jsonl 2> $out/ranks.err &&
timeout -k 10 200 bash scripts/loopback_probe.sh && mv gpurun_out/loopback.jsonl $out/loopback.jsonl &&
timeout -k 10 300 python scripts/workers_probe.py > $out/workers.jsonl 2> $out/workers.err
rc=$?
echo "exit $rc"
exit $rc
