# objCrop column pass: both halves' strip loads before the first barrier
# (lib_crp) vs per half (in-tree): objCrop tests on lib_crp, metric A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/crp
mkdir -p $O
FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_crp/libfpm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do
  for V in default crp; do
    if [ $V = default ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$V/libfpm_hip.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/m_$V$i.json 2> $O/m_$V$i.err || exit 1
    python3 -c "import json; d=json.load(open('$O/m_$V$i.json')); print('metric $V', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"
  done
done
