# general-path K4 batching + layout copy variants: tests, config 5 bench, setup A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_groups.py tests/test_gpu_configs.py -k "groups or config5 or fp16" -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head -20; tail -5 $O/t.log; exit 1; }
tail -2 $O/t.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_$i.json 2> $O/c5_$i.err || { echo "bench rc=$?"; tail -3 $O/c5_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$i.json')); print('c5', d['value'], d['ms_per_step'], d['led_ms_per_step'])"
done
bash tools/gpu/layout_ab.sh
