# A/B of library builds (tools/build_variant.sh) on the metric bench, after
# the fused-path parity tests of the default build.
#   VARIANTS="ilp memclause" TAG=v1 bash tools/gpu/variants.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-var}
mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
for V in base $VARIANTS; do
  if [ $V = base ]; then L=""; else L=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_var/$V/libfpm_hip.so; fi
  FPM_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline $BENCHARGS > $O/bench_$V.json 2> $O/bench_$V.err || { echo "BENCH $V rc=$?"; tail $O/bench_$V.err; exit 1; }
  FPM_HIP_LIB=$L FPM_STAMPS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline $BENCHARGS > /dev/null 2> $O/stamps_$V.err || { echo "STAMPS $V rc=$?"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$V.json')); print('$V', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"
  grep "fpm stamps" $O/stamps_$V.err | tail -1
done
