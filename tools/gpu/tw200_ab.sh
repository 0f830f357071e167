# Np 200 twiddle asm blocks (in-tree) vs one pmul per twiddle (lib_tw200s) on
# config 3; Np 256 blocks of five vs single (lib_tws) on the metric config
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tw200
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused_mr.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
VARS=tw200s BENCH_ARGS="--config c3" TAG=tw200/c3 bash tools/gpu/ab_multi.sh || exit 1
VARS=tws ROUNDS=2 TAG=tw200/metric bash tools/gpu/ab_multi.sh
