# patch groups on concurrent streams (general path): tests, then config 5
# bench for G = 1 / 2 / 4 with and without the iteration graph
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/groups
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_groups.py -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head -20; tail -5 $O/t.log; exit 1; }
tail -3 $O/t.log
for i in 1 2; do
  for V in ${VARS:-"FPM_PATCH_GROUPS=1" "FPM_PATCH_GROUPS=2" "FPM_PATCH_GROUPS=4" "FPM_PATCH_GROUPS=2 FPM_NO_GRAPH=1" "FPM_PATCH_GROUPS=8"}; do
    N=$(echo $V | tr ' =' '__')
    env $V timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/$N$i.json 2> $O/$N$i.err || { echo "$V rc=$?"; tail -3 $O/$N$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$N$i.json')); print('$V', d['value'], d['ms_per_step'], d['led_ms_per_step'])"
  done
done
