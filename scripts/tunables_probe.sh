# glibc malloc tunables A/B on the 1- and 8-queue thread fleet (scripts/pmu_probe.py --quick), r02l.
set -o pipefail
mkdir -p gpurun_out
for t in "" "glibc.malloc.tcache_count=1000" "glibc.malloc.arena_max=1" "glibc.malloc.tcache_count=0"; do
  GLIBC_TUNABLES="$t" timeout -k 10 120 python -u scripts/pmu_probe.py --quick >> gpurun_out/tunables.jsonl 2>> gpurun_out/tunables.err || exit 1
done
