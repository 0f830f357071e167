# full GPU suite on the in-tree build, then the layout copy with 8-byte
# quad-column LDS reads (in-tree) vs 2-byte reads (FPM_LAYOUT_U16=1):
# setup timing of the metric and config-3 benches, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/layq
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
for C in metric c3; do
  for i in 1 2 3; do
    for E in FPM_AB_NONE=1 FPM_LAYOUT_U16=1; do
      env $E timeout -k 10 200 python bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline > $O/${C}_${E%%=*}_$i.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.load(open('$O/${C}_${E%%=*}_$i.json')); print('$C', '$E', d['setup']['upload_and_permute_ms'], d['setup']['init_ms'], d['led_ms_per_step'])"
    done
  done
done
