set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03d}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 300 --timeout-method thread > $O/split_tests.log 2>&1 || { echo "SPLIT TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert|PASS" $O/split_tests.log | head -40; exit 1; }
tail -1 $O/split_tests.log
for T in 128 64 32; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --patches-total $T --no-cpu-baseline > $O/bench_pt$T.json 2> $O/bench_pt$T.err || { echo "BENCH pt$T rc=$?"; tail $O/bench_pt$T.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_pt$T.json')); print('patches-total $T', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['config']['kernel'])"
done
FPM_NO_DIST=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --patches-total 128 --no-cpu-baseline > $O/bench_pt128s.json 2> $O/bench_pt128s.err && python3 -c "import json; d=json.load(open('$O/bench_pt128s.json')); print('split patches-total 128', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['config']['kernel'])"
FPM_DIST=4 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --patches-total 32 --no-cpu-baseline > $O/bench_pt32d4.json 2> $O/bench_pt32d4.err && python3 -c "import json; d=json.load(open('$O/bench_pt32d4.json')); print('dist4 patches-total 32', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['config']['kernel'])"
for K in 2 4 8; do FPM_DIST=$K FPM_STAMPS=1 timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gather --patches-total $((256/K)) > $O/st$K.json 2> $O/st$K.err; grep "fpm stamps" $O/st$K.err; done
