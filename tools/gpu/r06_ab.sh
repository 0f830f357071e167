# Round 6 A/B: optional parity tests (TESTS=...), optional bit-identity
# (CMP=<lib name>), phase stamps (STAMPS=workloads), then alternating bench
# lines of the in-tree library ("new") against fpm-opencv_amd/lib_<v>/ for v
# in VARS, per workload in LINES; each line prints value, LED ms per step,
# objCrop ms per step, the in-kernel clock and kernel cycles per launch
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06ab}
mkdir -p $O
python3 tools/srchash.py > $O/srchash.txt
if [ -n "$TESTS" ]; then
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
if [ -n "$SMOKE" ]; then
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
fi
if [ -n "$CMP" ]; then
timeout -k 10 600 python tools/gpu/cmp_libs.py fpm-opencv_amd/lib/libfpm_hip.so fpm-opencv_amd/lib_$CMP/libfpm_hip.so > $O/cmp.txt 2>&1; rc=$?; tail -9 $O/cmp.txt; [ $rc -le 1 ] || exit 1
fi
args() { case $1 in metric) echo "";; pt128|pt128d2) echo "--patches-total 128";; pt64) echo "--patches-total 64";; pt32) echo "--patches-total 32";; c2) echo "--config c2";; c2np256) echo "--config c2 --np 256";; c3) echo "--config c3";; c5) echo "--config c5";; esac; }
# workload-specific environment (pt128d2: the 128-patch shard on the distributed kernel at 2 parts)
wenv() { case $1 in pt128d2) echo "FPM_DIST=2";; *) echo "FPM_X=0";; esac; }
show() { python3 -c "import json; d=json.load(open('$1')); print('$2', d['value'], d['led_ms_per_step'], d['objcrop_ms_per_step'], d.get('clock_mhz'), d.get('kernel_cycles_per_launch'))"; }
for w in ${STAMPS:-}; do
  for V in ${STLIBS:-new}; do
    if [ $V = new ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$V/libfpm_hip.so; fi
    env $(wenv $w) FPM_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gather $(args $w) > $O/st_${w}_$V.json 2> $O/st_${w}_$V.err || { echo "stamps $w $V rc=$?"; tail -3 $O/st_${w}_$V.err; exit 1; }
    echo "== stamps $w $V"; grep "fpm stamps" $O/st_${w}_$V.err | tail -2
  done
done
unset FPM_HIP_LIB
for i in $(seq 1 ${ROUNDS:-2}); do
  for w in ${LINES:-metric}; do
    for V in new $VARS; do
      if [ $V = new ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$V/libfpm_hip.so; fi
      env $(wenv $w) timeout -k 10 180 python bench.py ${AB_STEPS:---steps 20 --warmup 3} --no-cpu-baseline --no-gather $(args $w) > $O/${w}_$V$i.json 2> $O/${w}_$V$i.err || { echo "$w $V rc=$?"; tail -3 $O/${w}_$V$i.err; exit 1; }
      show $O/${w}_$V$i.json "$w $V"
    done
  done
done
