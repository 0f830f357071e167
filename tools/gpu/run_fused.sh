set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t3.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -30 gpurun_out/t3.log; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err || { echo "BENCH FAILED rc=$?"; tail gpurun_out/bench_fused.err; exit 1; }
cat gpurun_out/bench_fused.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_fused -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/prof_fused.log 2>&1 || echo "PROF rc=$?"
