# Bare TCP-loopback round trips (csrc/tools/loopback_probe.cc): N clients as threads of one
# process (also with a private fd table per thread) vs N processes, client i and its echo server on CCD i. Output: gpurun_out/loopback.jsonl
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BIN=kube_sqs_autoscaler_amd/ops/loopback_probe.bin
for round in 1 2 3; do
  for n in 1 2 4 8; do
    spec=$(python3 -c "
from kube_sqs_autoscaler_amd.utils.topology import llc_domains, physical_cores
d = llc_domains()
print(','.join(f'{physical_cores(d[i])[0][0]}:{physical_cores(d[i])[1][0]}' for i in range($n)))")
    for mode in threads threads-unshare procs; do
      timeout -k 5 60 $BIN $mode $n 20000 "$spec" | python3 -c "
import sys, json
rows = [json.loads(l) for l in sys.stdin]
print(json.dumps({'mode': '$mode', 'n': $n, 'round': $round, 'spec': '$spec', 'p50_ns': [r.get('p50_ns') for r in rows]}))" >> gpurun_out/loopback.jsonl || exit 1
    done
  done
done
