# small-patch fused kernel: its parity tests, configs 1/2, config-2 bench on both paths
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-small}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_small.py tests/test_gpu_configs.py -x -v -k "small or config1 or config2" --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert|rel" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { echo "BENCH c2 rc=$?"; tail $O/bench_c2.err; exit 1; }
FPM_NO_SMALL=1 timeout -k 10 300 python bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c2_general.json 2> $O/bench_c2g.err || { echo "BENCH c2 general rc=$?"; tail $O/bench_c2g.err; exit 1; }
for f in bench_c2 bench_c2_general; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('led_ms_per_step'), d.get('objcrop_ms_per_step'))"; done
