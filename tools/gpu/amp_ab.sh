# A/B of kernel variants built by tools/build_variant.sh (lib_var/NAME): full GPU
# tests on the default build, fused-path parity tests of each variant (a
# numerical failure there is reported, not fatal), then the metric bench and
# the config c2/c3 lines for the default build and each variant in VARIANTS.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
for v in ${VARIANTS}; do
  [ -n "$SKIP_TESTS" ] && break
  FPM_HIP_LIB=$PWD/fpm-opencv_amd/lib_var/$v/libfpm_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_small.py tests/test_gpu_fused_mr.py -q --timeout 240 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?
  echo "variant $v tests rc=$rc: $(tail -1 $O/tests_$v.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
done
for v in default ${VARIANTS}; do
  if [ $v = default ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$PWD/fpm-opencv_amd/lib_var/$v/libfpm_hip.so; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/m_$v.json 2> $O/m_$v.err || { echo "bench $v rc=$?"; tail $O/m_$v.err; exit 1; }
  if [ -z "$ONLY_M" ]; then
  timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline > $O/c3_$v.json 2> $O/c3_$v.err || { echo "c3 $v rc=$?"; tail $O/c3_$v.err; exit 1; }
  timeout -k 10 300 python bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline > $O/c2_$v.json 2> $O/c2_$v.err || { echo "c2 $v rc=$?"; tail $O/c2_$v.err; exit 1; }
  fi
  FS="m c3 c2"; [ -n "$ONLY_M" ] && FS=m
  for f in $FS; do python3 -c "import json; d=json.load(open('$O/${f}_$v.json')); print('$v $f', d['value'], d['ms_per_step'], d.get('led_ms_per_step'), d.get('objcrop_ms_per_step'))"; done
done
