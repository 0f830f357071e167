# slot update with the object / pupil coefficient chains side by side
# (in-tree) vs chained (lib_updchain): parity tests of the fused kernels, then
# metric, config 2, config 3 and 64-patch benches, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/updi
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_metric.py tests/test_gpu_configs.py tests/test_gpu_fused_s90.py tests/test_gpu_fused_mr.py tests/test_gpu_update_coef.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
VARS=updchain TAG=updi/metric bash tools/gpu/ab_multi.sh || exit 1
VARS=updchain ROUNDS=2 BENCH_ARGS="--config c2" TAG=updi/c2 bash tools/gpu/ab_multi.sh || exit 1
VARS=updchain ROUNDS=2 BENCH_ARGS="--config c3" TAG=updi/c3 bash tools/gpu/ab_multi.sh || exit 1
VARS=updchain ROUNDS=2 BENCH_ARGS="--patches 64" TAG=updi/pt64 bash tools/gpu/ab_multi.sh
