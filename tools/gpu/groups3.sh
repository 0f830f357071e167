# per-group graphs: tests, then config 5 for G = 1..4 with graphs and G = 2 direct
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/groups3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_groups.py tests/test_gpu_update_coef.py -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head -20; tail -5 $O/t.log; exit 1; }
tail -2 $O/t.log
for i in 1 2; do
  for V in "FPM_PATCH_GROUPS=1" "FPM_PATCH_GROUPS=2" "FPM_PATCH_GROUPS=3" "FPM_PATCH_GROUPS=4" "FPM_PATCH_GROUPS=2_FPM_NO_GRAPH=1"; do
    E=$(echo $V | sed 's/_FPM_NO/ FPM_NO/')
    env $E timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/$V$i.json 2> $O/$V$i.err || { echo "$V rc=$?"; tail -3 $O/$V$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$V$i.json')); print('$E', d['value'], d['ms_per_step'], d['led_ms_per_step'])"
  done
done
