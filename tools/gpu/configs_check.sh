# fp16-storage parity tests + auxiliary config measurements (c3, c5) + c5 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-cfg}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "C3 FAILED rc=$?"; tail $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
timeout -k 10 400 python bench.py --config c5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "C5 FAILED rc=$?"; tail $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
timeout -k 10 400 python bench.py --config c5 --patches 1 --steps 2 --warmup 1 > $O/bench_c5_b1.json 2> $O/bench_c5_b1.err || { echo "C5 B1 FAILED rc=$?"; tail $O/bench_c5_b1.err; exit 1; }
cat $O/bench_c5_b1.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 1 --warmup 0 > $O/prof_c5.log 2>&1 || { echo "PROF rc=$?"; exit 1; }
python3 tools/prof_summary.py $O/prof_c5 $O/kernel_stats_c5.csv fpm
