# Diagnostic: how the box's CPU share and placement affect multi-queue / multi-rank latency.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/place
mkdir -p $out
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os; print(len(os.sched_getaffinity(0)), sorted(os.sched_getaffinity(0))[:32])"; lscpu | grep -i "model name\|numa node\|socket\|thread"; } > $out/cpus.txt 2>&1
timeout -k 10 120 python bench.py --queues 8 --no-sweep > $out/q8_free.json 2> $out/q8_free.err &&
timeout -k 10 120 taskset -c 0-7 python bench.py --queues 8 --no-sweep > $out/q8_pin8.json 2> $out/q8_pin8.err &&
timeout -k 10 120 taskset -c 0-15 python bench.py --queues 8 --no-sweep > $out/q8_pin16.json 2> $out/q8_pin16.err &&
HIP_VISIBLE_DEVICES= timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 4 --steps 2000 --warmup 200 > $out/r4_cpu.json 2> $out/r4_cpu.err &&
HIP_VISIBLE_DEVICES= timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 8 --steps 2000 --warmup 200 > $out/r8_cpu.json 2> $out/r8_cpu.err
rc=$?
echo "exit $rc"
exit $rc
