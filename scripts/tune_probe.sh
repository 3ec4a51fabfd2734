set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./kube_sqs_autoscaler_amd/ops/tune_probe.bin > gpurun_out/tune_probe.jsonl 2> gpurun_out/tune_probe.err
