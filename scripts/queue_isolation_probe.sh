# Diagnostic: which in-process sharing raises multi-queue latency (fake servers vs logger).
# Interleaved repetitions, because single runs on a shared host vary by +-20 %.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${ISO_OUT:-iso}
mkdir -p $out
for rep in 1 2 3; do
  for cfg in "shared shared" "per-queue shared" "shared per-queue"; do
    set -- $cfg
    timeout -k 10 120 python bench.py --queues 8 --no-sweep --servers $1 --loggers $2 > $out/q8_$1_$2_r$rep.json 2> $out/q8_$1_$2_r$rep.err || exit $?
  done
done
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || exit $?
echo done
