# full GPU check of the tree: parity tests, smoke, default bench (with the CPU
# baseline leg), kernel-trace stats of the same bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-chk}
mkdir -p $O
lscpu > $O/lscpu.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED rc=$?"; tail $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED rc=$?"; tail $O/bench.err; exit 1; }
cat $O/bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "PROF rc=$?"; exit 1; }
python3 tools/prof_summary.py $O/prof $O/kernel_stats.csv fpm
