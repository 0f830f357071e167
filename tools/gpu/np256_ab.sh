# Np 256 kernel variant A/B: parity tests of the in-tree build, then metric /
# 128 / 64-patch benches against lib_<v> for v in VARS (default tws)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-tw5}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_metric.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
VARS="${VARS:-tws}" TAG=${TAG:-tw5}/metric bash tools/gpu/ab_multi.sh || exit 1
VARS="${VARS:-tws}" ROUNDS=2 BENCH_ARGS="--patches 128" TAG=${TAG:-tw5}/pt128 bash tools/gpu/ab_multi.sh || exit 1
VARS="${VARS:-tws}" ROUNDS=2 BENCH_ARGS="--patches 64" TAG=${TAG:-tw5}/pt64 bash tools/gpu/ab_multi.sh
