# The headline's run-to-run spread: ten `bench.py` runs with the driver's flags (no secondary
# rows) in a row on one box, each under its own time limit; the first failure ends the pass.
# OUT: where the runs go (default gpurun_out/r05l).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05l}
mkdir -p "$OUT"
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-sweep > "$OUT/headline_$i.json" 2> "$OUT/headline_$i.err" || exit $?
done
echo done
