# pass B: the younger waves stop claiming column blocks near the end
# (lib_ys2 / lib_ys4: none of the last 2 / 4 blocks) vs the in-tree build;
# parity tests on lib_ys4, then metric / config 3 / 128-patch A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ystop
mkdir -p $O
FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_ys4/libfpm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_fused_mr.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
VARS="ys2 ys4" TAG=ystop/metric bash tools/gpu/ab_multi.sh || exit 1
VARS="ys2 ys4" ROUNDS=2 BENCH_ARGS="--config c3" TAG=ystop/c3 bash tools/gpu/ab_multi.sh || exit 1
VARS="ys2 ys4" ROUNDS=2 BENCH_ARGS="--patches 128" TAG=ystop/pt128 bash tools/gpu/ab_multi.sh
