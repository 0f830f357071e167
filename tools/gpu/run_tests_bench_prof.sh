set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t2.log 2>&1 || { echo "TESTS FAILED rc=$?"; exit 1; }
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --path general > gpurun_out/bench_general.json 2> gpurun_out/bench_general.err || { echo "BENCH FAILED rc=$?"; exit 1; }
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_general -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --path general --no-cpu-baseline > gpurun_out/prof_general.log 2>&1 || echo "PROF rc=$?"
lscpu | head -20 > gpurun_out/lscpu.txt
