# Np 90 register-transform kernel: tests, then config 2 bench vs the generic small kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s90
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_s90.py tests/test_gpu_fused_small.py -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head -20; tail -5 $O/t.log; exit 1; }
tail -2 $O/t.log
for i in 1 2; do
  for V in "FPM_AB_NONE=1" "FPM_NO_S90=1"; do
    env $V timeout -k 10 300 python bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline > $O/c2_$V$i.json 2> $O/c2_$V$i.err || { echo "bench rc=$?"; tail -3 $O/c2_$V$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c2_$V$i.json')); print('$V', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['config']['kernel'])"
  done
done
