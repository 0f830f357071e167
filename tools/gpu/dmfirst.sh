# distributed mode: first-round measurement before sync 1 (in-tree) vs not (lib_var)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/dmfirst
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -q -k "dist" --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
BENCH_ARGS="--patches-total 64" TAG=dmfirst/pt64 bash tools/gpu/ab_lib.sh && BENCH_ARGS="--patches-total 32" TAG=dmfirst/pt32 bash tools/gpu/ab_lib.sh
