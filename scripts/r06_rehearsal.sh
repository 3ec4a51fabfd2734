# Round 6's GPU-box rehearsal of the driver's round-end runs: the GPU tests, smoke(), then the
# driver's exact bench command with its stdout cut to the driver's 8,000-character capture and
# parsed (scripts/check_bench_line.py), and a 2-rank gloo rehearsal of the multi-GPU line. Every
# step has its own time limit; the first failure ends the pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${1:-r06a}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest_gpu.log" 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 &&
timeout -k 10 700 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench.stdout" 2> "$out/bench.err" &&
cp gpurun_out/bench_detail.json "$out/bench_detail.json" &&
tail -c 8000 "$out/bench.stdout" | python3 scripts/check_bench_line.py > "$out/bench_line_check.json" &&
timeout -k 10 300 python3 bench.py --gpus 2 --steps 200 --warmup 20 --no-sweep --rehearse-shared-gpus \
    --detail-out "$out/bench_ranks2_detail.json" > "$out/bench_ranks2.stdout" 2> "$out/bench_ranks2.err" &&
tail -c 8000 "$out/bench_ranks2.stdout" | python3 scripts/check_bench_line.py --no-sweep > "$out/bench_ranks2_line_check.json"
rc=$?
echo "exit $rc"
exit $rc
