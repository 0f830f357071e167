# Np 256 register path (np256.hip): its tests, the c2np256 bench line of each
# variant (new = in-tree lib; old = FPM_NO_REG256=1; other names = lib_<name>)
# alternating, and a kernel trace of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06n}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_np256.py ${EXTRA_TESTS} > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert|rel L2" $O/tests.log | head -30; exit 1; }
grep -E "passed|failed|rel L2" $O/tests.log | tail -8
venv() {
  case $1 in
    new) echo "FPM_X=1";;
    old) echo "FPM_NO_REG256=1";;
    g1) echo "FPM_PATCH_GROUPS=1";;
    g2) echo "FPM_PATCH_GROUPS=2";;
    g3) echo "FPM_PATCH_GROUPS=3";;
    g4) echo "FPM_PATCH_GROUPS=4";;
    *) echo "FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_$1/libfpm_hip.so";;
  esac
}
for R in $(seq 1 ${ROUNDS:-1}); do
for V in ${VARS:-new old}; do
  env $(venv $V) timeout -k 10 300 python bench.py --config c2 --np 256 --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline ${BARGS} > $O/c2np256_${V}$R.json 2> $O/c2np256_${V}$R.err || { echo "bench $V rc=$?"; tail -3 $O/c2np256_${V}$R.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2np256_${V}$R.json')); print('$V', d['value'], d['ms_per_step'], d['led_ms_per_step'], d['objcrop_ms_per_step'])"
done
done
[ -n "$NOTRACE" ] && exit 0
for V in ${VARS:-new old}; do
  env $(venv $V) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_$V -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c2 --np 256 --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_$V.log 2>&1 || { echo "kernel trace $V rc=$?"; tail -5 $O/kt_$V.log; exit 1; }
  find $O/kt_$V -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_c2np256_$V.csv \;
  find $O/kt_$V -name "*kernel_trace.csv" -delete
  echo "== $V"
  python3 -c "
import csv
for r in csv.DictReader(open('$O/kernel_stats_c2np256_$V.csv')):
    n = r['Name'].replace('(anonymous namespace)::', '')
    if int(r['Calls']) >= 100 and 'at::' not in n:
        print('  %-40s %5s %8.2f us' % (n.split('(')[0], r['Calls'], float(r['AverageNs']) / 1e3))"
done
