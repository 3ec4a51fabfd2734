# Rehearse the driver's 1/2/4/8-rank bench on one box with the ranks on the CPU (gloo): this
# workload's scaling is CPU-side (one autoscaler + its fakes per rank), and the GPU box has only
# one card. Each N runs bench.py under torch.distributed.run exactly as the driver does, once
# per placement given (default: rank-l3 and kernel).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export CUDA_VISIBLE_DEVICES="" HIP_VISIBLE_DEVICES=""
port=29611
for pl in ${@:-rank-l3 kernel}; do
  for n in 1 2 4 8; do
    port=$((port + 1))
    timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus $n --steps 2000 --warmup 200 --no-sweep --placement $pl \
      > gpurun_out/ranks_${pl}_n$n.json 2> gpurun_out/ranks_${pl}_n$n.err || exit 1
  done
done
