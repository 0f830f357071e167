# persistent pipelined layout copy (in-tree) vs one block per strip
# (FPM_LAYOUT_SIMPLE=1): layout tests, then setup timing of metric / c3
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/laypipe
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_torch_interop.py tests/test_gpu_metric.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
for C in metric c3; do
  for i in 1 2 3; do
    for E in FPM_AB_NONE=1 FPM_LAYOUT_SIMPLE=1; do
      env $E timeout -k 10 200 python bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline > $O/${C}_${E%%=*}_$i.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.load(open('$O/${C}_${E%%=*}_$i.json')); print('$C', '$E', d['setup']['upload_and_permute_ms'], d['setup']['init_ms'])"
    done
  done
done
