# first-round measurement prefetch (in-tree) vs none (lib_var): smoke parity then metric A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/mfirst
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_metric.py tests/test_gpu_split.py -x -q -k "one_workgroup or split2 or bench" --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
TAG=mfirst/ab bash tools/gpu/ab_lib.sh
