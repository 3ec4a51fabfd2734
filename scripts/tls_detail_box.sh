# TLS vs plain per-phase probe (scripts/tls_detail.py), twice, on the GPU box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/tls_detail.py > gpurun_out/tls_detail2.jsonl 2> gpurun_out/tls_probe2.err &&
timeout -k 10 200 python -u scripts/tls_detail.py >> gpurun_out/tls_detail2.jsonl 2>> gpurun_out/tls_probe2.err
