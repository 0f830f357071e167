# Round 4 A/B runner: optional GPU tests (TESTS = pytest arguments), then for
# every workload in WORKLOADS ("name:bench args;name:bench args") the in-tree
# library against fpm-opencv_amd/lib_$VAR/libfpm_hip.so, alternating REPS
# times on one box (value, ms per step, LED ms, objCrop ms).
#   TAG=r04c VAR=v2 TESTS="tests/test_gpu_parity.py -k objcrop" WORKLOADS="c3:--config c3" bash tools/gpu/ab_run.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}
mkdir -p $O
python3 tools/srchash.py > $O/srchash.txt
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
  tail -1 $O/tests.log
fi
IFS=';' read -ra WL <<< "${WORKLOADS:-metric:}"
for i in $(seq 1 ${REPS:-2}); do
  for W in "${WL[@]}"; do
    N=${W%%:*}; A=${W#*:}; E=FPM_AB_NONE=1
    case "$A" in FPM_*) E=${A%% *}; A=${A#* };; esac  # "name:FPM_X=1 --args": an environment setting for both
    for V in cur $VAR; do
      if [ $V = cur ]; then unset FPM_HIP_LIB; else export FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$V/libfpm_hip.so; fi
      env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-gather $A > $O/${N}_$V$i.json 2> $O/${N}_$V$i.err || { echo "$N $V rc=$?"; tail -3 $O/${N}_$V$i.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${N}_$V$i.json')); print('$N $V', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'], d['config']['kernel'])"
    done
  done
done
unset FPM_HIP_LIB
