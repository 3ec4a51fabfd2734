# TLS vs plain: per-phase probe, then user-mode sampling profiles of one plain and one TLS queue.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/pmu_sample
timeout -k 10 200 python -u scripts/tls_detail.py > gpurun_out/tls_detail.jsonl 2> gpurun_out/tls_probe.err &&
timeout -k 10 200 python -u scripts/pmu_sample.py --tls > gpurun_out/pmu_sample_tls.log 2>&1 &&
timeout -k 10 200 python -u scripts/pmu_sample.py > gpurun_out/pmu_sample_plain.log 2>&1
