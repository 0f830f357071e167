# L 4096 objCrop (config 5): parity tests, then config 5 with the in-tree
# library and with the variant library lib_$VAR, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-c4k}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_np1024.py tests/test_gpu_configs.py -k "objcrop_l4096 or config5" -x -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert|Timeout" $O/tests.log | head -30; exit 1; }
grep -E "passed|six-step|rel L2" $O/tests.log | tail -12
for i in 1 2; do
  for V in cur $VAR; do
    if [ $V = cur ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$V/libfpm_hip.so; fi
    timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_$V$i.json 2> $O/c5_$V$i.err || { echo "bench $V rc=$?"; tail -5 $O/c5_$V$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c5_$V$i.json')); print('c5 $V', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"
  done
done
unset FPM_HIP_LIB
