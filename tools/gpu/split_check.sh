# split mode (two workgroups per patch): its tests first, then the fused parity
# and config tests (small batches run split), then the config-4 shard bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-split}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 120 --timeout-method thread > $O/split_tests.log 2>&1 || { echo "SPLIT TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert" $O/split_tests.log | head -30; tail -5 $O/split_tests.log; exit 1; }
tail -1 $O/split_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --patches-total 128 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_shard128.json 2> $O/c4s.err || { echo "c4 shard rc=$?"; tail $O/c4s.err; exit 1; }
FPM_NO_SPLIT=1 timeout -k 10 300 python bench.py --patches-total 128 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_shard128_nosplit.json 2> $O/c4n.err || { echo "c4 nosplit rc=$?"; tail $O/c4n.err; exit 1; }
for f in c4_shard128 c4_shard128_nosplit; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"; done
FPM_STAMPS=1 timeout -k 10 240 python bench.py --patches-total 128 --steps 1 --warmup 0 --no-cpu-baseline 2>&1 >/dev/null | grep "fpm stamps" > $O/split_stamps.txt || true
cat $O/split_stamps.txt
