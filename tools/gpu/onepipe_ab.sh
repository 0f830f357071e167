# Np 256: fifteen twiddles in one asm block (lib_one), software-pipelined
# amplitude step (lib_pipe), both (lib_onepipe) vs the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/onepipe
mkdir -p $O
FPM_HIP_LIB=$GRAFT_REPO_ROOT/fpm-opencv_amd/lib_onepipe/libfpm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_metric.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
VARS="one pipe onepipe" TAG=onepipe/metric bash tools/gpu/ab_multi.sh || exit 1
VARS="onepipe" ROUNDS=2 BENCH_ARGS="--patches 64" TAG=onepipe/pt64 bash tools/gpu/ab_multi.sh
