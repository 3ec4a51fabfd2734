# Sweep kernel: exactness tests, timed run, then PMC passes (--pmc only with --kernel-trace/--stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 &&
timeout -k 10 300 python -m pytest tests/test_gpu.py -x -q -k sweep > gpurun_out/pytest_sweep.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o sweep -- python3 scripts/sweep_bench.py > gpurun_out/prof_sweep.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc -o sweep -- python3 scripts/sweep_bench.py > gpurun_out/pmc_sweep.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc2 -o sweep -- python3 scripts/sweep_bench.py > gpurun_out/pmc2_sweep.log 2>&1
