# Np 200 fused kernel: its parity tests (+ metric parity), config-3 bench line, stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-c3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_mr.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { echo "c3 rc=$?"; tail $O/c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3.json')); print('c3', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"
FPM_STAMPS=1 timeout -k 10 300 python bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline 2>&1 >/dev/null | grep stamps || true
