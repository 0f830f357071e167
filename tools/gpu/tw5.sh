# twiddle multiplies in asm blocks of five (in-tree) vs one asm fma per
# twiddle (lib_tws): Np 256 parity tests, then metric / 128 / 64-patch A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tw5
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_metric.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
VARS=tws TAG=tw5/metric bash tools/gpu/ab_multi.sh || exit 1
VARS=tws ROUNDS=2 BENCH_ARGS="--patches 128" TAG=tw5/pt128 bash tools/gpu/ab_multi.sh || exit 1
VARS=tws ROUNDS=2 BENCH_ARGS="--patches 64" TAG=tw5/pt64 bash tools/gpu/ab_multi.sh
