# Np 1024 persistent chain kernel: parity tests, then config 5 with and without it
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-chain1}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_np1024.py -x -v -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert|Timeout" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_chain.json 2> $O/c5_chain.err || { echo "bench chain rc=$?"; tail -5 $O/c5_chain.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5_chain.json')); print('chain', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['roofline']['kernel'])"
FPM_NO_CHAIN=1 timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_perled.json 2> $O/c5_perled.err || { echo "bench perled rc=$?"; tail -5 $O/c5_perled.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5_perled.json')); print('per-LED', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['roofline']['kernel'])"
