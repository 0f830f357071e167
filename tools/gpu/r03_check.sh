# round-3 check: split/metric tests first, then the whole -m gpu suite, the
# headline bench line and the strong-scaling shards; one box call
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_metric.py -x -v -s --timeout 300 --timeout-method thread > $O/new_tests.log 2>&1 || { echo "NEW TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert|rel L2" $O/new_tests.log | head -40; tail -5 $O/new_tests.log; exit 1; }
grep -E "rel L2|passed|failed" $O/new_tests.log | tail -30
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "BENCH rc=$?"; tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('metric', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'], d['roofline']['frac'])"
for T in 128 64 32; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --patches-total $T --no-cpu-baseline > $O/bench_pt$T.json 2> $O/bench_pt$T.err || { echo "BENCH pt$T rc=$?"; tail $O/bench_pt$T.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_pt$T.json')); print('patches-total $T', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['config']['workgroups_per_patch'])"
done
(rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || true)
grep -o "TCC_EA0_[A-Z0-9_]*" $O/list_avail.txt | sort -u | tr '\n' ' ' || true
