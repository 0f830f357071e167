# full GPU test suite (one pytest process) + one bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-gt}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH rc=$?"; tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"
