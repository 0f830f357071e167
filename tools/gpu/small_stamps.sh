# small-patch kernel at config 2: parity tests, bench line, phase stamps from the
# FPM_SMALL_STAMPS=1 variant (tools/build_variant.sh sstamps -DFPM_SMALL_STAMPS=1).
# Stamp indices: 0 gather, 7 row IDFT, 1 transpose in, 10 col IDFT, 2 amplitude,
# 8 col DFT, 3 transpose out, 9 row DFT, 4 update, 5 max, 6 pupil
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ss}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_small.py tests/test_gpu_configs.py -x -q -k "small or config1 or config2" --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert|rel" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { echo "BENCH c2 rc=$?"; tail $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print('c2', d['value'], d['ms_per_step'], d.get('led_ms_per_step'), d.get('objcrop_ms_per_step'))"
if [ -f fpm-opencv_amd/lib_var/sstamps/libfpm_hip.so ]; then
FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_var/sstamps/libfpm_hip.so FPM_STAMPS=1 timeout -k 10 240 python bench.py --config c2 --steps 1 --warmup 0 --no-cpu-baseline > $O/c2s.json 2> $O/c2s.err || { echo "rc=$?"; tail $O/c2s.err; exit 1; }
grep "fpm stamps" $O/c2s.err | head -1
fi
