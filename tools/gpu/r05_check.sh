# Round 5 check: the whole -m gpu suite (one pytest process), the no-flag bench
# line, and one line per workload whose kernel this round works on.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05a}
mkdir -p $O
python3 tools/srchash.py > $O/srchash.txt
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread --durations 15 ${TESTS:-} > $O/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
line() {  # name, env, bench args
  env $2 timeout -k 10 180 python bench.py --no-cpu-baseline --no-gather $3 > $O/$1.json 2> $O/$1.err || { echo "$1 rc=$?"; tail -3 $O/$1.err; return 1; }
  echo "== $1: $(python3 -c "import json; d=json.load(open('$O/$1.json')); print(d['value'], d['led_ms_per_step'], d['objcrop_ms_per_step'], d['config']['kernel'], d['roofline'].get('frac'))")"
}
for w in ${LINES:-metric pt64 pt32 c2 c3 c5}; do
  case $w in
    metric) line metric "FPM_X=0" "" ;;
    pt128) line pt128 "FPM_X=0" "--patches-total 128" ;;
    pt64) line pt64 "FPM_X=0" "--patches-total 64" ;;
    pt32) line pt32 "FPM_X=0" "--patches-total 32" ;;
    c2) line c2 "FPM_X=0" "--config c2" ;;
    c3) line c3 "FPM_X=0" "--config c3" ;;
    c5) line c5 "FPM_X=0" "--config c5" ;;
  esac || exit 1
done
