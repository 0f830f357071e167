# Np 200 kernel with two barriers fewer per LED (in-tree) vs before (lib_var)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/mrbar
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_mr.py "tests/test_gpu_configs.py::test_config3_dogstomach_literal_256_patches" -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
BENCH_ARGS="--config c3" TAG=mrbar/ab bash tools/gpu/ab_lib.sh
