# batched slot updates (in-tree) vs one slot at a time (lib_updser): parity
# tests of every kernel that changed, then metric / 128 / 64-patch and
# config 3 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/upd
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_metric.py tests/test_gpu_fused_mr.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
VARS=updser TAG=upd/metric bash tools/gpu/ab_multi.sh || exit 1
VARS=updser ROUNDS=2 BENCH_ARGS="--patches 64" TAG=upd/pt64 bash tools/gpu/ab_multi.sh || exit 1
VARS=updser ROUNDS=2 BENCH_ARGS="--config c3" TAG=upd/c3 bash tools/gpu/ab_multi.sh
