# Probe kernel tuning: variant sweep + the shipped probe on the same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 &&
timeout -k 10 120 ./kube_sqs_autoscaler_amd/ops/tune_probe.bin > gpurun_out/tune_probe.jsonl 2> gpurun_out/tune_probe.err &&
timeout -k 10 120 python scripts/probe_bench.py > gpurun_out/probe_bench.jsonl 2> gpurun_out/probe_bench.err
