# the whole -m gpu suite + smoke, one pytest process
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-full}
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/tests.log | head -30; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE rc=$?"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
