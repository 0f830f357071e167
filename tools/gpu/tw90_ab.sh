# Np 90 twiddles in asm pairs (in-tree) vs one pmul each (lib_tw90s):
# Np 90 tests, then config 2 benches, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tw90
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_s90.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
VARS=tw90s ROUNDS=3 BENCH_ARGS="--config c2" TAG=tw90/c2 bash tools/gpu/ab_multi.sh
