# Round 5 A/B: the in-tree library against lib_base (the committed tree) --
# bit-identity (cmp_libs), phase stamps and alternating bench lines per
# workload; optional parity tests first (TESTS=...)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05ab}
mkdir -p $O
python3 tools/srchash.py > $O/srchash.txt
BASE=${BASE:-base}
if [ -n "$TESTS" ]; then
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
if [ -z "$NO_CMP" ]; then
timeout -k 10 600 python tools/gpu/cmp_libs.py fpm-opencv_amd/lib/libfpm_hip.so fpm-opencv_amd/lib_$BASE/libfpm_hip.so > $O/cmp.txt 2>&1; rc=$?; cat $O/cmp.txt | tail -8; [ $rc -le 1 ] || exit 1
fi
args() { case $1 in metric) echo "";; pt128|pt128d2) echo "--patches-total 128";; pt64) echo "--patches-total 64";; pt32) echo "--patches-total 32";; c2) echo "--config c2";; c3) echo "--config c3";; c5) echo "--config c5";; esac; }
# workload-specific environment (pt128d2: the 128-patch shard on the distributed kernel at 2 parts)
wenv() { case $1 in pt128d2) echo "FPM_DIST=2";; *) echo "FPM_X=0";; esac; }
for w in ${STAMPS:-}; do
  for V in ${STLIBS:-new $BASE}; do
    if [ $V = new ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$V/libfpm_hip.so; fi
    env $(wenv $w) FPM_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gather $(args $w) > $O/st_${w}_$V.json 2> $O/st_${w}_$V.err || { echo "stamps $w $V rc=$?"; tail -3 $O/st_${w}_$V.err; exit 1; }
    echo "== stamps $w $V"; grep "fpm stamps" $O/st_${w}_$V.err | tail -2
  done
done
unset FPM_HIP_LIB
for i in $(seq 1 ${ROUNDS:-2}); do
  for w in ${LINES:-metric}; do
    for V in new $BASE $VARS; do
      if [ $V = new ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$V/libfpm_hip.so; fi
      env $(wenv $w) timeout -k 10 180 python bench.py ${AB_STEPS:---steps 20 --warmup 3} --no-cpu-baseline --no-gather $(args $w) > $O/${w}_$V$i.json 2> $O/${w}_$V$i.err || { echo "$w $V rc=$?"; tail -3 $O/${w}_$V$i.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${w}_$V$i.json')); print('$w $V', d['value'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"
    done
  done
done
