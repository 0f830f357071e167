# tests + bench + kernel-trace stats + HBM counter passes, one box call
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "BENCH FAILED rc=$?"; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo "PROF rc=$?"; exit 1; }
bash tools/gpu/prof_counters.sh
